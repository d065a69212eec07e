"""Block-cyclic row sharding of one frame across ranks.

Rows are grouped in blocks of ``band_rows`` (8); block b goes to rank
b % band_count, which balances sky rows against geometry rows.  Each rank
renders its blocks into a compact buffer of ``band_local_rows`` rows (all
ranks equal, padded), the buffers are gathered to rank 0 back to back, and
``assemble`` (host restatement of the HIP kernel behind rt_assemble_bands)
puts rows back in image order.  Pixels are independent
(RayTracingSetup.cs:288-301), so the assembled frame is bit-identical to a
single-GPU frame.
"""
from __future__ import annotations

import numpy as np


def band_local_rows(res_y: int, band_count: int, band_rows: int = 8) -> int:
    """Rows of every rank's compact buffer (== rt_band_rows_local)."""
    if res_y <= 0:
        return 0
    if band_count <= 1:
        return res_y
    blocks = -(-res_y // band_rows)
    slots = -(-blocks // band_count)
    return slots * band_rows


def band_global_rows(res_y: int, band_index: int, band_count: int, band_rows: int = 8) -> np.ndarray:
    """Global row of each local row of rank band_index (-1 = padding)."""
    n = band_local_rows(res_y, band_count, band_rows)
    if band_count <= 1:
        return np.arange(n)
    ly = np.arange(n)
    blk = ly // band_rows
    gy = (blk * band_count + band_index) * band_rows + (ly - blk * band_rows)
    return np.where(gy < res_y, gy, -1)


def assemble(gathered: np.ndarray, res_y: int, band_rows: int = 8) -> np.ndarray:
    """(band_count, local_rows, W, C) gathered shards -> (res_y, W, C) image."""
    band_count, local_rows = gathered.shape[:2]
    if band_count == 1:
        return gathered[0, :res_y]
    gy = np.arange(res_y)
    blk = gy // band_rows
    band = blk % band_count
    slot = blk // band_count
    ly = slot * band_rows + (gy - blk * band_rows)
    return gathered[band, ly]


def assemble_frames(gathered: np.ndarray, res_y: int, frames: int, band_rows: int = 8) -> np.ndarray:
    """(band_count, frames * local_rows, W, C): the shards of `frames` frames,
    each rank's stacked frame after frame (one gather per frame group) ->
    (frames, res_y, W, C).  local_rows is a multiple of band_rows, so the
    stack is the block-cyclic shard of one tall image of frames * local_rows *
    band_count rows in which frame j starts at row j * local_rows * band_count:
    one reassembly (bench.py: rt_assemble_bands over the tall image) serves
    the whole group."""
    band_count, tall_local = gathered.shape[:2]
    local_rows = tall_local // frames
    assert local_rows * frames == tall_local and (band_count == 1 or local_rows % band_rows == 0)
    span = local_rows * band_count
    tall = assemble(gathered, frames * span, band_rows)
    return tall.reshape(frames, span, *tall.shape[1:])[:, :res_y]
