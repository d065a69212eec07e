"""MaxReflectionBounces beyond the library's 32-entry fold stack.

The reference's MaxReflectionBounces is an unbounded int
(RayTracingSetup.cs:23, tested at :358 `bounce < MaxReflectionBounces`).
A mirror corridor (scenes.mirror_corridor) sends rays tens to hundreds of
bounces deep; frames must equal the brute-force oracle (whose Shade is the
literal recursion) within 1e-4 per channel (observed: bit-identical) with
identical primary/shadow/reflection ray counts, for every render path the
flags name (deep frames always run the megakernel's deep-chain instance)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _check(rt, gpu_ctx, orc, fr, flags=0, build=0):
    gpu_ctx.set_scene(fr.scene, build)
    img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags))
    ref, counts = orc.render(fr)
    err = float(np.max(np.abs(img.astype(np.float64) - ref.astype(np.float64))))
    assert err <= TOL, f"{fr.name} spp{fr.spp} flags {flags}: max err {err}"
    got = (st.primary_rays, st.shadow_rays, st.reflection_rays)
    want = (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"])
    assert got == want, f"{fr.name}: ray counts {got} != oracle {want}"
    return counts


@pytest.mark.parametrize("depth", [32, 33, 40, 64, 300])
@pytest.mark.parametrize("spp", [1, 4])
def test_corridor_depth(rt, gpu_ctx, orc, depth, spp):
    fr = rt.scenes.mirror_corridor(depth, spp=spp)
    counts = _check(rt, gpu_ctx, orc, fr)
    if depth > 32:  # the scene really has chains deeper than the fold stack
        shallow = orc.render(rt.scenes.mirror_corridor(32, spp=spp))[1]
        assert counts["reflection_rays"] > shallow["reflection_rays"]


@pytest.mark.parametrize("flags_name", ["RT_FLAG_COUNT_TESTS", "RT_FLAG_PACKET", "RT_FLAG_WAVEFRONT",
                                        "RT_FLAG_ROW_ORDER", "RT_FLAG_OUT_RGB32F"])
def test_corridor_paths(rt, gpu_ctx, orc, flags_name):
    fr = rt.scenes.mirror_corridor(48)
    flags = getattr(rt.abi, flags_name)
    if flags_name == "RT_FLAG_OUT_RGB32F":
        gpu_ctx.set_scene(fr.scene)
        img, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags))
        ref, _ = orc.render(fr)
        assert np.array_equal(img.view(np.uint32), ref[..., :3].copy().view(np.uint32))
        return
    _check(rt, gpu_ctx, orc, fr, flags=flags)


@pytest.mark.parametrize("build", [0, 1])
def test_corridor_mesh_walls_and_lbvh(rt, gpu_ctx, orc, build):
    """The walls as one SceneMesh (mesh-AABB gate, negated normals), both BVH builders."""
    _check(rt, gpu_ctx, orc, rt.scenes.mirror_corridor(70, loose=False), build=build)


def test_corridor_16spp(rt, gpu_ctx, orc):
    """16 spp frames normally take the all-packet levels kernel; deep ones the megakernel."""
    _check(rt, gpu_ctx, orc, rt.scenes.mirror_corridor(40, res=(8, 6), spp=16))


def test_corridor_bands(rt, gpu_ctx, orc):
    """A block-cyclic shard of a deep frame equals the same rows of the whole frame."""
    fr = rt.scenes.mirror_corridor(50, res=(24, 40))
    ref, _ = orc.render(fr)
    gpu_ctx.set_scene(fr.scene)
    n, rows = 3, 8
    for b in range(n):
        img, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, band_index=b, band_count=n, band_rows=rows))
        ys = [y for y in range(fr.plane.ResolutionY) if (y // rows) % n == b]
        assert np.max(np.abs(img[:len(ys)] - ref[ys])) <= TOL  # shards are padded to whole blocks
