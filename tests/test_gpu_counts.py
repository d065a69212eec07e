"""Canonical test counts: the GPU counting launch
(RT_FLAG_COUNT_TESTS, per-lane traversal of csrc/traverse.h with the exact
node test) must report exactly the box / triangle / sphere / shading counts of
the CPU oracle's walk of the same exported 4-wide tree (oracle/rt_oracle.c
bvh4_query, a step-for-step restatement of that traversal: same node test,
same child order, same any-hit early exit, same mesh-gate re-evaluation) —
plus the reference's ray counts and the same pixels.  These counts price
`roofline.logical_bytes_per_launch` in bench.py; the loop they count is
Scene.IntersectRay (Data/Objects/Scene.cs:43-122) accelerated by the tree.

Covered: C2, C3 and C5 reduced frames, the mirror corridor past the 32-level
fold stack (the deep-chain instance re-walks segments without recounting
them), a fuzz scene with every primitive kind, both BVH builders."""
import numpy as np
import pytest

from test_gpu_fuzz import random_frame

pytestmark = pytest.mark.gpu

KEYS = ("primary_rays", "shadow_rays", "reflection_rays", "box_tests", "triangle_tests", "sphere_tests",
        "shading_fetches")


def gpu_counts(st):
    return {"primary_rays": st.primary_rays, "shadow_rays": st.shadow_rays, "reflection_rays": st.reflection_rays,
            "box_tests": st.box_tests, "triangle_tests": st.triangle_tests, "sphere_tests": st.sphere_tests,
            "shading_fetches": st.shading_fetches}


def check_counts(rt, ctx, orc, fr, build):
    ctx.set_scene(fr.scene, build)
    img, st = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS))
    nodes, tris, sphs = ctx.export_bvh()
    b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
    try:
        W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
        ref, want = b4.render_pixels(np.arange(W * H, dtype=np.int32))
    finally:
        b4.close()
    got = gpu_counts(st)
    assert np.array_equal(img.reshape(-1, 4).view(np.uint32), ref.view(np.uint32)), fr.name
    bad = {k: (got[k], want[k]) for k in KEYS if got[k] != want[k]}
    assert not bad, f"{fr.name} build {build}: GPU counting launch vs oracle walk (got, want): {bad}"
    return got


@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("name,res", [("C2", (96, 54)), ("C3", (120, 68)), ("C5", (40, 24)), ("demo", None),
                                      ("C1", (64, 64))])
def test_counting_launch_equals_oracle_walk(rt, gpu_ctx, orc, name, res, build):
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    c = check_counts(rt, gpu_ctx, orc, fr, build)
    assert c["box_tests"] > 0 and c["shading_fetches"] > 0


@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("depth", [8, 40])
def test_counts_deep_mirror_corridor(rt, gpu_ctx, orc, depth, build):
    fr = rt.scenes.mirror_corridor(depth, loose=False)
    c = check_counts(rt, gpu_ctx, orc, fr, build)
    assert c["reflection_rays"] > 0


@pytest.mark.parametrize("seed", [3, 11])
def test_counts_fuzz(rt, gpu_ctx, orc, seed):
    check_counts(rt, gpu_ctx, orc, random_frame(rt, seed), 0)
