"""Device-side mesh extraction (rt_set_scene_source / rt_update_mesh_transforms,
SURVEY §8(f) rank 2).  The reference re-extracts every SceneMesh each Update()
(RayTracingSetup.cs:120-128,159-169; SceneMesh.cs:11-53): vertices through
localToWorldMatrix.MultiplyPoint3x4, Mesh.AABB over all vertices, triangles in
index order, normals -Triangle.Normal.  The device extraction must give the
same bytes as the host restatement (scene.py Mesh.from_vertices), so frames
and hits equal the host-extracted scene's and the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _counts(st):
    return (st.primary_rays, st.shadow_rays, st.reflection_rays)


def test_demo_cube_extracted_on_device(gpu_ctx, rt):
    """The reference demo (RayTracing.unity) with its Cube extracted on the
    device renders the committed golden frame bit for bit."""
    import os
    fr = rt.make("demo")
    base = rt.scenes.without_meshes(fr.scene)
    gpu_ctx.set_scene_source(base, [rt.scenes.demo_cube_source()])
    img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "frames.npz"))
    assert _same(img[..., :3].copy(), g["demo"])
    assert _counts(st) == tuple(g["demo_counts"])
    info = gpu_ctx.scene_info()
    assert info["build"] == 1 and info["primitives"] == 12 + 2 + 1


def _mixed_sources(rt):
    """Knot mesh under a rotation + non-uniform scale, a few cubes, an empty
    mesh and a mesh with vertices but no triangles."""
    S = rt.scenes
    verts, idx = S.torus_knot(segments=96, sides=24)
    q = np.array([0.2, 0.3, -0.1, 0.927], np.float32)
    q /= np.float32(np.linalg.norm(q))
    srcs = [rt.MeshSource(verts, idx, rt.scene.quaternion_trs((0.1, -0.2, 0.2), q, (1.3, 0.8, 1.1)), S.KNOT_MAT)]
    cv, ci = S.unit_cube()
    for k in range(5):
        m = rt.scene.quaternion_trs((-0.6 + 0.3 * k, -0.7, -0.4), S.yaw_quaternion(0.4 * k), (0.15, 0.25, 0.15))
        srcs.append(rt.MeshSource(cv, ci, m, S.MIRROR if k == 2 else S.BOX_MAT))
    eye = np.eye(4, dtype=np.float32)
    srcs.append(rt.MeshSource(np.zeros((0, 3), np.float32), np.zeros(0, np.int32), eye, S.BOX_MAT))
    srcs.append(rt.MeshSource(cv, np.zeros(0, np.int32), eye, S.BOX_MAT))
    return srcs


def test_mixed_sources_equal_host_extraction(gpu_ctx, rt, orc):
    fr0 = rt.make("C2").with_resolution(160, 90)
    base = rt.scenes.without_meshes(fr0.scene)
    srcs = _mixed_sources(rt)
    host = rt.scenes.extracted(fr0.with_(scene=base), srcs)
    gpu_ctx.set_scene_source(base, srcs)
    a, sa = gpu_ctx.render(host.camera, host.plane, rt.frame_params(host))
    gpu_ctx.set_scene(host.scene, 0)
    b, sb = gpu_ctx.render(host.camera, host.plane, rt.frame_params(host))
    assert _same(a, b) and _counts(sa) == _counts(sb)
    ref, counts = orc.render(host)
    assert float(np.max(np.abs(a - ref))) <= TOL
    assert _counts(sa) == (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"])


def test_big_mesh_aabb_in_parts(gpu_ctx, rt, orc):
    """C3's 35k-vertex knot as one source mesh: its Mesh.AABB is reduced over
    18 parts of 2,048 vertices (scene_xform.hip k_aabb_parts) and must give
    the host extraction's frame and the oracle's."""
    S = rt.scenes
    fr0 = rt.make("C3").with_resolution(96, 54)
    base = S.without_meshes(fr0.scene)
    verts, idx = S.torus_knot()
    assert len(verts) > 16 * 2048
    srcs = [rt.MeshSource(verts, idx, np.eye(4, dtype=np.float32), S.KNOT_MAT)]
    host = S.extracted(fr0.with_(scene=base), srcs)
    gpu_ctx.set_scene_source(base, srcs)
    a, sa = gpu_ctx.render(host.camera, host.plane, rt.frame_params(host))
    gpu_ctx.set_scene(host.scene, 0)
    b, sb = gpu_ctx.render(host.camera, host.plane, rt.frame_params(host))
    assert _same(a, b) and _counts(sa) == _counts(sb)
    ref, counts = orc.render(host)
    assert float(np.max(np.abs(a - ref))) <= TOL


def test_intersect_on_device_extracted_geometry(gpu_ctx, rt, orc):
    """Hit distances are bit-exact, so the device's world-space vertices equal
    the host's MultiplyPoint3x4 results."""
    fr0 = rt.make("C2")
    base = rt.scenes.without_meshes(fr0.scene)
    srcs = _mixed_sources(rt)
    host = rt.scenes.extracted(fr0.with_(scene=base), srcs)
    gpu_ctx.set_scene_source(base, srcs)
    rng = np.random.default_rng(3)
    n = 6000
    o = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d.astype(np.float32)], 1)
    hits = gpu_ctx.intersect_rays(rays)
    ref = orc.intersect(host.scene, rays)
    assert (ref["type"] == 3).sum() > 500
    for f in ("type", "index"):
        assert np.array_equal(hits[f], ref[f]), f
    mesh = ref["type"] == 3
    assert np.array_equal(hits["mesh_index"][mesh], ref["mesh_index"][mesh])
    assert np.array_equal(hits["distance"].view(np.uint32), ref["distance"].view(np.uint32))


def test_animated_transform_updates(gpu_ctx, rt, orc):
    """Per-frame rt_update_mesh_transforms: each frame equals the oracle on
    the host-extracted scene with that frame's matrices."""
    fr, srcs, mats = rt.scenes.instanced_hall(400, res=(96, 54), spp=1, bounces=4)
    gpu_ctx.set_scene_source(fr.scene, srcs)
    for k, t in enumerate((0.0, 0.37, 1.1, 2.5)):
        m = mats(t)
        if k:
            gpu_ctx.update_mesh_transforms(m)
        img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
        host = rt.scenes.extracted(fr, srcs, m)
        ref, counts = orc.render(host)
        assert float(np.max(np.abs(img - ref))) <= TOL, t
        assert _counts(st) == (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), t
        info = gpu_ctx.scene_info()
        assert info["build_ms"] > 0.0


def test_update_equals_fresh_source_scene(gpu_ctx, rt):
    """An updated scene renders exactly like a scene set from scratch with
    the same matrices (the update path reuses device state correctly)."""
    fr, srcs, mats = rt.scenes.instanced_hall(2000, res=(320, 180), spp=1, bounces=8)
    gpu_ctx.set_scene_source(fr.scene, srcs)
    gpu_ctx.update_mesh_transforms(mats(0.8))
    a, sa = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    tree_a = gpu_ctx.export_bvh()
    moved = [rt.MeshSource(s.Vertices, s.Indices, m, s.MaterialData) for s, m in zip(srcs, mats(0.8))]
    gpu_ctx.set_scene_source(fr.scene, moved)
    b, sb = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    assert _same(a, b) and _counts(sa) == _counts(sb)
    # the update folds the scene box and its padding on the device
    # (k_scene_box); the host computes them for a fresh scene: same bits,
    # hence the same sort keys, padded boxes and tree
    for x, y in zip(tree_a, gpu_ctx.export_bvh()):
        assert np.array_equal(x, y)


def test_source_errors(gpu_ctx, rt):
    S = rt.scenes
    fr = rt.make("C1").with_resolution(8, 8)
    cv, ci = S.unit_cube()
    bad = ci.copy()
    bad[5] = 24  # out of range
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.set_scene_source(fr.scene, [rt.MeshSource(cv, bad, np.eye(4, dtype=np.float32), S.BOX_MAT)])
    assert e.value.status == rt.abi.RT_E_SCENE
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.set_scene_source(fr.scene, [rt.MeshSource(cv, ci[:7], np.eye(4, dtype=np.float32), S.BOX_MAT)])
    assert e.value.status == rt.abi.RT_E_SCENE
    gpu_ctx.set_scene(fr.scene)
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.update_mesh_transforms(np.eye(4, dtype=np.float32)[None])
    assert e.value.status == rt.abi.RT_E_STATE
    gpu_ctx.set_scene_source(fr.scene, [rt.MeshSource(cv, ci, np.eye(4, dtype=np.float32), S.BOX_MAT)])
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.update_mesh_transforms(np.stack([np.eye(4, dtype=np.float32)] * 2))
    assert e.value.status == rt.abi.RT_E_INVALID


# ---- RT_BUILD_SAH_REFIT (rt_set_scene_source_ex): host SAH tree once, device refits ----

def test_refit_updates_equal_oracle(gpu_ctx, rt, orc):
    """Refitted trees (same topology, new boxes and records every update)
    render each frame like the oracle on the host-extracted scene."""
    fr, srcs, mats = rt.scenes.instanced_hall(400, res=(96, 54), spp=1, bounces=4)
    gpu_ctx.set_scene_source(fr.scene, srcs, build=rt.abi.RT_BUILD_SAH_REFIT)
    assert gpu_ctx.scene_info()["build"] == rt.abi.RT_BUILD_SAH_REFIT
    for k, t in enumerate((0.0, 0.37, 1.1, 2.5)):
        m = mats(t)
        if k:
            gpu_ctx.update_mesh_transforms(m)
        img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
        ref, counts = orc.render(rt.scenes.extracted(fr, srcs, m))
        assert float(np.max(np.abs(img - ref))) <= TOL, t
        assert _counts(st) == (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), t


def test_refit_equals_rebuilt_frames(rt):
    """The knot spinning about its centre (the shim's rebuild loop): a
    refitting context and a rebuilding (LBVH) context give the same frames
    bit for bit, frame after frame, mixed mesh and loose geometry included."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from rebuild_bench import c3_sources
    base, srcs, mats = c3_sources(rt)
    base = base.with_resolution(320, 180)
    a, b = rt.Context(), rt.Context()
    try:
        a.set_scene_source(base.scene, srcs, build=rt.abi.RT_BUILD_SAH_REFIT)
        b.set_scene_source(base.scene, srcs)
        for k in range(6):
            if k:
                m = mats(0.3 * k)
                a.update_mesh_transforms(m)
                b.update_mesh_transforms(m)
            ia, sa = a.render(base.camera, base.plane, rt.frame_params(base))
            ib, sb = b.render(base.camera, base.plane, rt.frame_params(base))
            assert _same(ia, ib) and _counts(sa) == _counts(sb), k
    finally:
        a.close()
        b.close()


def test_refit_large_motion_rebuilds(gpu_ctx, rt, orc):
    """Meshes scattered far from where the tree was built (the refitted
    tree's area explodes, so the update rebuilds it on the host) and then
    moved again: frames still equal the oracle."""
    fr, srcs, mats = rt.scenes.instanced_hall(200, res=(64, 36), spp=1, bounces=2)
    gpu_ctx.set_scene_source(fr.scene, srcs, build=rt.abi.RT_BUILD_SAH_REFIT)
    m0 = mats(0.0)
    rng = np.random.default_rng(5)
    for step in range(3):
        m = m0.copy()
        perm = rng.permutation(len(m))
        m[:, :3, 3] = m0[perm, :3, 3]  # every box jumps to another box's place
        gpu_ctx.update_mesh_transforms(m)
        img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
        ref, counts = orc.render(rt.scenes.extracted(fr, srcs, m))
        assert float(np.max(np.abs(img - ref))) <= TOL, step
        assert _counts(st) == (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), step


def test_refit_rejects_unknown_build(gpu_ctx, rt):
    fr, srcs, _ = rt.scenes.instanced_hall(8, res=(16, 16), spp=1, bounces=1)
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.set_scene_source(fr.scene, srcs, build=rt.abi.RT_BUILD_SAH_HOST)
    assert e.value.status == rt.abi.RT_E_INVALID
