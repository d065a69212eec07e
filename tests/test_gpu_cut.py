"""The camera packets' top-level cut start (packet.h cut_select, trace.hip
build_cut_kernel): a tile's camera packet starts from the cut entries its
widened frustum touches, and waiting entries are re-tested against each lane's
closest hit when popped.  Only the visiting order may change, so frames must
be bit-identical with the cut switched off (RT_FLAG_NO_CUT, every packet from the
root) and equal to the oracle — including scenes far from the origin (the
frustum test's slack), cameras inside the geometry, partial edge tiles, split
waves (longest-first quarter/sixteenth waves of small shards), row bands and
row slabs, and the device-built trees."""

import numpy as np
import pytest

from test_gpu_fuzz import random_frame

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _render(ctx, rt, fr, build=0, cut=True, **kw):
    if not cut:
        kw["flags"] = kw.get("flags", 0) | rt.abi.RT_FLAG_NO_CUT
    return ctx.render(fr.camera, fr.plane, rt.frame_params(fr, **kw))


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _translated(rt, fr, off):
    """The frame with every position moved by `off` (float32 adds, the camera
    too): the same picture far from the origin."""
    import copy

    o = np.asarray(off, np.float32)
    sc = copy.deepcopy(fr.scene)
    td = sc.TriangleData
    if len(td.Triangles):
        td.Triangles = (td.Triangles + o).astype(np.float32)
    for m in sc.Meshes:
        m.Triangles = (m.Triangles + o).astype(np.float32)
        m.AABB = (m.AABB + o).astype(np.float32)
    if len(sc.SphereData.Spheres):
        sc.SphereData.Spheres[:, :3] = (sc.SphereData.Spheres[:, :3] + o).astype(np.float32)
    if len(sc.PointLights):
        sc.PointLights[:, :3] = (sc.PointLights[:, :3] + o).astype(np.float32)
    cam = fr.camera.__class__(**{**fr.camera.__dict__,
                                 "Position": tuple((np.asarray(fr.camera.Position, np.float32) + o).tolist())})
    return fr.with_(scene=sc, camera=cam)


CASES = [("C3", (96, 54), 4), ("C3", (61, 37), 1), ("C2", (80, 45), 4), ("C5", (48, 27), 4), ("demo", None, 1),
         ("C1", (70, 50), 1)]


@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("name,res,spp", CASES)
def test_cut_equals_root_start_and_oracle(gpu_ctx, rt, orc, name, res, spp, build):
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=spp)
    gpu_ctx.set_scene(fr.scene, build)
    a, sa = _render(gpu_ctx, rt, fr, build)
    b, sb = _render(gpu_ctx, rt, fr, build, cut=False)
    assert _same(a, b), f"{name}: cut start changed the frame"
    assert (sa.primary_rays, sa.shadow_rays, sa.reflection_rays) == (sb.primary_rays, sb.shadow_rays,
                                                                       sb.reflection_rays)
    ref, counts = orc.render(fr)
    assert float(np.nanmax(np.abs(a.astype(np.float64) - ref))) <= TOL


@pytest.mark.parametrize("off", [(1.0e4, -3.0e3, 2.5e4), (-6.5e4, 0.0, 0.0)])
@pytest.mark.parametrize("seed", range(6))
def test_cut_far_from_origin(gpu_ctx, rt, orc, seed, off):
    fr = _translated(rt, random_frame(rt, 500 + seed, res=(48, 36), spp=4 if seed % 2 else 1, bounces=seed % 4),
                     off)
    gpu_ctx.set_scene(fr.scene, 0)
    a, _ = _render(gpu_ctx, rt, fr)
    b, _ = _render(gpu_ctx, rt, fr, cut=False)
    assert _same(a, b)
    ref, _ = orc.render(fr)
    err = np.abs(a.astype(np.float64) - ref.astype(np.float64))
    assert float(np.nanmax(err)) <= TOL


def test_cut_camera_inside_geometry(gpu_ctx, rt, orc):
    """The corridor: the camera inside long wall boxes (entries whose boxes
    contain the camera position)."""
    fr = rt.make("C3").with_resolution(64, 40)
    cam = fr.camera.__class__(**{**fr.camera.__dict__, "Position": (0.05, -0.1, 0.1)})  # inside the knot's box
    fr = fr.with_(camera=cam)
    gpu_ctx.set_scene(fr.scene, 0)
    a, _ = _render(gpu_ctx, rt, fr)
    b, _ = _render(gpu_ctx, rt, fr, cut=False)
    assert _same(a, b)
    ref, _ = orc.render(fr)
    assert float(np.nanmax(np.abs(a.astype(np.float64) - ref))) <= TOL


@pytest.mark.parametrize("band_rows", [8, 2, 3])
def test_cut_row_bands(gpu_ctx, rt, band_rows):
    """Row bands of 8 rows (cut on: 4-row tiles lie in one block) and of 2 / 3
    rows (a tile spans blocks: cut off) reassemble to the whole frame."""
    fr = rt.make("C3").with_resolution(96, 56)
    gpu_ctx.set_scene(fr.scene, 0)
    whole, _ = _render(gpu_ctx, rt, fr)
    n = 3
    rows = fr.plane.ResolutionY
    img = np.zeros_like(whole)
    for bi in range(n):
        part, _ = _render(gpu_ctx, rt, fr, band_index=bi, band_count=n, band_rows=band_rows)
        for k in range(part.shape[0]):
            blk, r = divmod(k, band_rows)
            gy = (blk * n + bi) * band_rows + r
            if gy < rows:
                img[gy] = part[k]
    assert _same(img, whole)


def test_cut_split_waves(gpu_ctx, rt):
    """Small frames split their slowest tiles into quarter and sixteenth
    waves (partial lanes): the second frame (measured order) equals the
    first and the root-start frame."""
    fr = rt.make("C3").with_resolution(160, 96)
    gpu_ctx.set_scene(fr.scene, 0)
    a, _ = _render(gpu_ctx, rt, fr)
    b, _ = _render(gpu_ctx, rt, fr)
    c, _ = _render(gpu_ctx, rt, fr, cut=False)
    assert _same(a, b) and _same(a, c)
