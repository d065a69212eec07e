"""On-device BVH build (rt_set_scene_ex(..., RT_BUILD_LBVH_GPU), SURVEY §8(f)
rank 1): the reference rebuilds its Scene every Update()
(RayTracingSetup.cs:120-128), so the drop-in must rebuild per frame on the
GPU.  The BVH only accelerates Scene.IntersectRay (Scene.cs:43-122), so every
answer must equal the brute-force oracle exactly, and frames must be
bit-identical to the host-SAH build."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4
LBVH = 1   # RT_BUILD_LBVH_GPU (collapsed to 4-wide nodes)
LBVH2 = 2  # RT_BUILD_LBVH_GPU_BVH2 (the same tree, 2-wide)
BUILDS = [LBVH, LBVH2]


def _frame(ctx, rt, fr, build):
    ctx.set_scene(fr.scene, build)
    return ctx.render(fr.camera, fr.plane, rt.frame_params(fr))


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_default_build_is_the_device_lbvh(gpu_ctx, rt):
    """rt_set_scene (no builder named) builds the 4-wide device LBVH; the frame
    equals the host SAH tree's bit for bit."""
    fr = rt.make("C2").with_resolution(160, 90)
    gpu_ctx.set_scene(fr.scene)
    info = gpu_ctx.scene_info()
    assert info["build"] == LBVH and info["bvh_width"] == 4
    a, sa = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    gpu_ctx.set_scene(fr.scene, 0)
    b, sb = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    assert _same(a, b)
    assert (sa.primary_rays, sa.shadow_rays, sa.reflection_rays) == (sb.primary_rays, sb.shadow_rays,
                                                                     sb.reflection_rays)


def test_scene_info(gpu_ctx, rt):
    fr = rt.make("C3")
    gpu_ctx.set_scene(fr.scene, 0)
    sah = gpu_ctx.scene_info()
    gpu_ctx.set_scene(fr.scene, LBVH)
    lb = gpu_ctx.scene_info()
    gpu_ctx.set_scene(fr.scene, LBVH2)
    lb2 = gpu_ctx.scene_info()
    n = fr.scene.triangle_count + len(fr.scene.SphereData.Spheres)
    assert sah["build"] == 0 and sah["bvh_width"] == 4 and sah["primitives"] == n and sah["build_ms"] == 0.0
    assert lb2["build"] == 2 and lb2["bvh_width"] == 2 and lb2["primitives"] == n and lb2["nodes"] == n - 1
    # even-depth 2-wide nodes become 4-wide nodes; small subtrees become leaves
    assert lb["build"] == 1 and lb["bvh_width"] == 4 and lb["primitives"] == n
    assert 1 <= lb["nodes"] < (n - 1) / 2
    for i in (lb, lb2):
        assert 0.0 < i["build_ms"] < i["total_ms"]


@pytest.mark.parametrize("build", BUILDS)
@pytest.mark.parametrize("name", ["C2", "C3", "C5"])
def test_full_frame_equals_sah(gpu_ctx, rt, name, build):
    """Full-size BASELINE frames: LBVH == SAH bit for bit (same ray counts)."""
    fr = rt.make(name)
    a, sa = _frame(gpu_ctx, rt, fr, 0)
    b, sb = _frame(gpu_ctx, rt, fr, build)
    assert _same(a, b)
    assert (sa.primary_rays, sa.shadow_rays, sa.reflection_rays) == (sb.primary_rays, sb.shadow_rays,
                                                                     sb.reflection_rays)


@pytest.mark.parametrize("build", BUILDS)
def test_intersect_rays_exact_lbvh(gpu_ctx, rt, orc, build):
    for name in ("demo", "C2", "C3", "C5"):
        fr = rt.make(name)
        gpu_ctx.set_scene(fr.scene, build)
        rng = np.random.default_rng(12)
        n = 4000 if name != "C5" else 1500
        o = rng.uniform(-1.2, 1.2, (n, 3)).astype(np.float32)
        if name == "demo":
            o *= 30
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        d[: n // 10, 1] = 0.0
        rays = np.concatenate([o, d.astype(np.float32)], 1)
        hits = gpu_ctx.intersect_rays(rays)
        ref = orc.intersect(fr.scene, rays)
        for f in ("type", "index"):
            assert np.array_equal(hits[f], ref[f]), (name, f)
        mesh = ref["type"] == 3
        assert np.array_equal(hits["mesh_index"][mesh], ref["mesh_index"][mesh]), name
        assert np.array_equal(hits["distance"].view(np.uint32), ref["distance"].view(np.uint32)), name


def test_dynamic_rebuild_per_frame(gpu_ctx, rt, orc):
    """An animated scene (objects move every frame, UpdateScene each Update):
    each frame is rebuilt on the device, reusing its buffers, and equals the
    oracle; shrinking and growing the scene between frames is fine."""
    base = rt.make("C2").with_resolution(96, 54)
    for k in range(6):
        sc = rt.scenes._c2_scene(with_boxes=(k % 3 != 2))
        ang = 0.7 * k
        sc.add_sphere_r2((0.4 * np.cos(ang), -0.1 + 0.1 * k, 0.3 * np.sin(ang)), 0.3 * 0.3, rt.scenes.MIRROR)
        for j in range(k):  # growing sphere count
            sc.add_sphere_r2((-0.6 + 0.2 * j, 0.6, -0.5), 0.05 * 0.05, rt.scenes.BLUE_PLASTIC)
        sc.PointLights = base.scene.PointLights
        sc.AmbientLight = base.scene.AmbientLight
        fr = base.with_(scene=sc)
        img, st = _frame(gpu_ctx, rt, fr, LBVH)
        ref, counts = orc.render(fr)
        assert float(np.max(np.abs(img - ref))) <= TOL, k
        assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (
            counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), k


@pytest.mark.parametrize("build", BUILDS)
def test_degenerate_scenes(gpu_ctx, rt, orc, build):
    """Morton-code collisions (identical centroids), a single primitive, a
    one-triangle mesh, zero-area triangles, a huge-coordinate scene."""
    S = rt.Scene
    fr0 = rt.make("C1").with_resolution(40, 30)
    mats = fr0.scene.SphereData.Materials
    scenes = []
    # 300 identical spheres plus 200 identical triangles: every key collides
    a = S()
    for i in range(300):
        a.add_sphere_r2((0.1, -0.2, 0.3), 0.2, mats[i % 2])
    tri = np.array([[[-0.5, -0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.5, 0.5]]], np.float32)
    a.add_triangles(np.repeat(tri, 200, 0), [mats[1]] * 200)
    scenes.append(a)
    # single sphere; single loose triangle; one mesh with one triangle
    b = S()
    b.add_sphere_r2((0.0, 0.0, 0.0), 0.25, mats[1])
    scenes.append(b)
    c = S()
    c.add_triangles(tri, [mats[1]])
    scenes.append(c)
    d = S()
    d.add_mesh(rt.Mesh.from_vertices(tri.reshape(-1, 3), [0, 1, 2], mats[1]))
    scenes.append(d)
    # zero-area triangles among normal ones
    e = S()
    z = np.array([[[0.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]],
                  [[-0.3, 0.0, 0.2], [0.3, 0.0, 0.2], [0.6, 0.0, 0.2]]], np.float32)
    e.add_triangles(np.concatenate([z, tri]), [mats[0]] * 3)
    scenes.append(e)
    # big coordinates: a far plane of spheres
    f = S()
    for i in range(64):
        f.add_sphere_r2((1.0e4 * (i % 8 - 3.5), 1.0e4 * (i // 8 - 3.5), 5.0e4), 1.0e7, mats[i % 2])
    scenes.append(f)
    for i, sc in enumerate(scenes):
        sc.PointLights = fr0.scene.PointLights
        sc.AmbientLight = fr0.scene.AmbientLight
        fr = fr0.with_(scene=sc)
        img, st = _frame(gpu_ctx, rt, fr, build)
        ref, counts = orc.render(fr)
        assert float(np.max(np.abs(img - ref))) <= TOL, i
        assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (
            counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), i
        img2, _ = _frame(gpu_ctx, rt, fr, 0)
        assert _same(img, img2), i


def test_rebuild_is_deterministic(gpu_ctx, rt):
    """The radix sort is stable and Karras' split is a pure function of the
    sorted keys, so two builds give the same tree; the frames are equal."""
    fr = rt.make("C3").with_resolution(320, 180)
    a, _ = _frame(gpu_ctx, rt, fr, LBVH)
    b, _ = _frame(gpu_ctx, rt, fr, LBVH)
    assert _same(a, b)


@pytest.mark.parametrize("build", [0] + BUILDS)
def test_degenerate_rays(gpu_ctx, rt, orc, build):
    """NaN, infinite and zero-direction rays: the traversal terminates (unused
    child slots lead to a sentinel leaf, never back to the root) and the
    answers equal the brute-force oracle."""
    fr = rt.make("C2")
    gpu_ctx.set_scene(fr.scene, build)
    rng = np.random.default_rng(5)
    n = 512
    o = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[0:64] = np.nan
    o[64:128, 1] = np.nan
    d[128:192] = 0.0
    d[192:256] = [np.inf, 0.0, 0.0]
    o[256:320] = [0.0, 0.0, 0.0]
    d[256:320, 0] = 0.0
    d[256:320, 2] = 0.0
    rays = np.concatenate([o, d.astype(np.float32)], 1).astype(np.float32)
    hits = gpu_ctx.intersect_rays(rays)
    ref = orc.intersect(fr.scene, rays)
    for f in ("type", "index"):
        assert np.array_equal(hits[f], ref[f]), f
    hit = ref["type"] != 0
    assert np.array_equal(hits["distance"][hit].view(np.uint32), ref["distance"][hit].view(np.uint32))
