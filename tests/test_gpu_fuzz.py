"""Randomised parity: seeded random scenes (loose triangles, spheres, meshes
with transforms, mirrors, specular materials, several lights, an ambient
light) rendered on the GPU with both BVH builders and compared with the
brute-force oracle — frame values within 1e-4 (observed: bit-identical) and
identical ray counts; plus random-ray closest-hit queries, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _material(rng, rt, mirror_p=0.25):
    return rt.MaterialData(
        DiffuseReflectance=tuple(rng.uniform(0, 1, 3)),
        AmbientReflectance=tuple(rng.uniform(0, 0.3, 3)),
        MirrorReflectance=tuple(rng.uniform(0, 1, 3)),
        SpecularReflectance=tuple(rng.uniform(0, 1, 3) * (rng.uniform() < 0.5)),
        PhongExponent=float(rng.choice([0.0, 1.0, 8.0, 50.0, rng.uniform(0, 200)])),
        IsMirror=bool(rng.uniform() < mirror_p))


def random_frame(rt, seed, res=(40, 30), spp=1, bounces=3):
    rng = np.random.default_rng(seed)
    S = rt.scenes
    sc = rt.Scene()
    n_tri = int(rng.integers(0, 40))
    if n_tri:
        tris = rng.uniform(-1.5, 1.5, (n_tri, 3, 3)).astype(np.float32)
        sc.add_triangles(tris, [_material(rng, rt) for _ in range(n_tri)])
    for _ in range(int(rng.integers(0, 6))):
        c = rng.uniform(-1.2, 1.2, 3)
        sc.add_sphere_r2(c, float(rng.uniform(0.01, 0.4)), _material(rng, rt))
    cv, ci = S.unit_cube()
    for _ in range(int(rng.integers(0, 5))):
        q = rng.normal(size=4).astype(np.float32)
        q /= np.float32(np.linalg.norm(q))
        m = rt.scene.quaternion_trs(rng.uniform(-1, 1, 3), q, rng.uniform(0.1, 0.8, 3))
        sc.add_mesh(rt.Mesh.from_vertices(cv, ci, _material(rng, rt), m))
    if rng.uniform() < 0.5:
        v, i = S.torus_knot(segments=24, sides=8, scale=float(rng.uniform(0.1, 0.3)))
        sc.add_mesh(rt.Mesh.from_vertices(v, i, _material(rng, rt)))
    for _ in range(int(rng.integers(0, 4))):
        sc.add_point_light(rng.uniform(-2, 2, 3), float(rng.uniform(0.5, 20.0)))
    sc.AmbientLight = rng.uniform(0, 20, 3).astype(np.float32)
    cam = S.CameraData(Position=(float(rng.uniform(-0.3, 0.3)), float(rng.uniform(-0.3, 0.3)), -3.4))
    plane = S.ImagePlane(res[0], res[1], 1.0, float(rng.uniform(0.3, 0.9)), float(rng.uniform(0.3, 0.6)))
    bg = tuple(rng.uniform(0, 1, 3)) + (1.0,)
    return S.Frame(f"fuzz{seed}", sc, cam, plane, background=bg, max_bounces=bounces, spp=spp)


@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("seed", range(40))
def test_random_scene_frames(gpu_ctx, rt, orc, seed, build):
    fr = random_frame(rt, seed, spp=4 if seed % 3 == 0 else 1, bounces=int(seed % 5))
    gpu_ctx.set_scene(fr.scene, build)
    img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    ref, counts = orc.render(fr)
    err = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    assert np.array_equal(np.isnan(img), np.isnan(ref))
    assert float(np.nanmax(err)) <= TOL, (seed, float(np.nanmax(err)))
    assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (
        counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]), seed


@pytest.mark.parametrize("seed", range(12))
def test_random_scene_hits(gpu_ctx, rt, orc, seed):
    fr = random_frame(rt, 100 + seed)
    gpu_ctx.set_scene(fr.scene, seed % 2)
    rng = np.random.default_rng(seed)
    n = 3000
    o = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d.astype(np.float32)], 1)
    hits = gpu_ctx.intersect_rays(rays)
    ref = orc.intersect(fr.scene, rays)
    for f in ("type", "index"):
        assert np.array_equal(hits[f], ref[f]), (seed, f)
    mesh = ref["type"] == 3
    assert np.array_equal(hits["mesh_index"][mesh], ref["mesh_index"][mesh])
    assert np.array_equal(hits["distance"].view(np.uint32), ref["distance"].view(np.uint32))
