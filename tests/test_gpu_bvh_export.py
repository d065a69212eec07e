"""rt_export_bvh: the 4-wide BVH as it lies in HBM, and the CPU traversal of
that very tree (oracle Bvh4Scene, the bench's "bvh_same_tree" CPU leg).

The exported records must describe a tree whose CPU traversal gives the
brute-force oracle's frames bit for bit (Scene.IntersectRay,
Data/Objects/Scene.cs:43-122, with the tree only accelerating it), and the
counts must agree with rt_get_scene_info — for the host SAH build and the
device LBVH build."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("name,res", [("C2", (96, 54)), ("C3", (120, 68)), ("C5", (64, 36)), ("demo", None)])
def test_exported_tree_renders_like_brute_force(rt, gpu_ctx, orc, name, res, build):
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    gpu_ctx.set_scene(fr.scene, build)
    info = gpu_ctx.scene_info()
    nodes, tris, sphs = gpu_ctx.export_bvh()
    assert len(nodes) == 128 * info["nodes"]
    n_tri = len(fr.scene.TriangleData.Triangles) + sum(len(m.Triangles) for m in fr.scene.Meshes)
    assert len(tris) == 48 * (n_tri + 1)  # + the sentinel record
    assert len(sphs) == 32 * len(fr.scene.SphereData.Spheres)
    # every triangle rank appears exactly once in the leaf-ordered records
    ranks = np.frombuffer(tris.tobytes(), np.int32).reshape(-1, 12)[:-1, 9]
    assert np.array_equal(np.sort(ranks[ranks >= 0]), np.sort(np.concatenate(
        [np.arange(sum(len(m.Triangles) for m in fr.scene.Meshes)),
         np.arange(len(fr.scene.TriangleData.Triangles)) + sum(len(m.Triangles) for m in fr.scene.Meshes)
         + len(fr.scene.SphereData.Spheres)])))
    b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
    try:
        W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
        idx = np.arange(W * H, dtype=np.int32)
        got, cg = b4.render_pixels(idx)
        ref, cr = orc.render_pixels(fr, idx)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), name
        for k in ("primary_rays", "shadow_rays", "reflection_rays"):
            assert cg[k] == cr[k], k
        # the tree is a real acceleration: far fewer primitive tests than the scan
        assert cg["triangle_tests"] <= cr["triangle_tests"]
    finally:
        b4.close()


def test_export_needs_a_four_wide_tree(rt, gpu_ctx):
    fr = rt.make("C2").with_resolution(32, 18)
    gpu_ctx.set_scene(fr.scene, rt.abi.RT_BUILD_LBVH_GPU_BVH2)
    with pytest.raises(rt.RtError):
        gpu_ctx.export_bvh()
    gpu_ctx.set_scene(fr.scene)
