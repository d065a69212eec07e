"""Multi-rank row sharding on CPU (gloo, world_size 2 and 3): every rank
renders its block-cyclic row shard, shards are gathered to rank 0 and
reassembled; the result must be bit-identical to the single-rank frame.
The per-rank renderer here is the CPU oracle (the HIP renderer is covered by
tests/test_gpu_parity.py::test_determinism_and_bands on the GPU box); what
this test pins is the distributed logic bench.py uses: band partition,
gather, reassembly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _rt_pkg
        rt = _rt_pkg.load()
        orc = _rt_pkg.load_oracle()
        from unity_raytracer_amd import bands
        fr = rt.make("C2").with_resolution(40, 37).with_(spp=4)
        W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
        rows = bands.band_global_rows(H, rank, world, 8)
        local = np.zeros((len(rows), W, 4), np.float32)
        live = rows >= 0
        idx = (rows[live][:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.int32)
        px, counts = orc.render_pixels(fr, idx, threads=1)
        local[live] = px.reshape(-1, W, 4)
        t = torch.from_numpy(local)
        gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, gathered, dst=0)
        rays = torch.tensor([counts["primary_rays"] + counts["shadow_rays"] + counts["reflection_rays"]],
                            dtype=torch.int64)
        dist.all_reduce(rays)
        if rank == 0:
            img = bands.assemble(torch.stack(gathered).numpy(), H, 8)
            full, fc = orc.render(fr, threads=2)
            q.put((bool(np.array_equal(img.view(np.uint32), full.view(np.uint32))),
                   int(rays.item()), fc["primary_rays"] + fc["shadow_rays"] + fc["reflection_rays"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_gather_bit_identical(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    same, rays, full_rays = q.get(timeout=10)
    assert same
    assert rays == full_rays  # sharding neither drops nor duplicates rays


def test_band_partition_covers_rows_once(rt):
    from unity_raytracer_amd import bands
    lib = rt.load_library()
    for H in (1, 7, 8, 9, 123, 1080, 2160):
        for n in (1, 2, 3, 4, 8):
            loc = bands.band_local_rows(H, n, 8)
            assert loc == lib.rt_band_rows_local(H, 0, n, 8)
            allrows = np.concatenate([bands.band_global_rows(H, r, n, 8) for r in range(n)])
            live = allrows[allrows >= 0]
            assert np.array_equal(np.sort(live), np.arange(H))
            g = np.stack([np.where(bands.band_global_rows(H, r, n, 8) >= 0,
                                   bands.band_global_rows(H, r, n, 8), -1) for r in range(n)])
            img = bands.assemble(g[..., None, None], H, 8)
            assert np.array_equal(img[:, 0, 0], np.arange(H))


def test_frame_group_reassembly_is_per_frame_reassembly(rt):
    """bench.py gathers a group of frames per collective (each rank's shards
    stacked frame after frame) and reassembles the group as one tall image;
    every frame must come out as its own per-frame reassembly would."""
    from unity_raytracer_amd import bands
    rng = np.random.default_rng(7)
    for H in (37, 1080):
        for n in (1, 2, 3, 8):
            for G in (1, 2, 4):
                loc = bands.band_local_rows(H, n, 8)
                shards = rng.integers(0, 1 << 30, size=(G, n, loc, 3, 2), dtype=np.int64)
                group = np.concatenate([shards[j] for j in range(G)], axis=1)  # (n, G*loc, W, C)
                got = bands.assemble_frames(group, H, G, 8)
                for j in range(G):
                    assert np.array_equal(got[j], bands.assemble(shards[j], H, 8)), (H, n, G, j)
