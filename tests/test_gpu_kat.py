"""The hand-derived known answers of tests/golden/kat.json through the HIP
path (rt_intersect_rays = Scene.IntersectRay, Data/Objects/Scene.cs:43-122).

tests/test_oracle.py checks these cases against the CPU oracle only; here
each case becomes a one-primitive scene on the device, so the reference's
only known answer — RayTracerTests.cs:11-26, ray (0,0,0)->(1,0,0) against a
sphere at (300,0,0) with r^2 = 1: t = 299 exactly — and the triangle and
slab edge cases run through the gfx950 kernels (both BVH builders):

* sphere cases: the sphere alone (RMath.RaySphereIntersection, RMath.cs:81-108,
  behind the Scene.AABB gate of its own box, Scene.cs:54);
* triangle cases: the triangle as a loose triangle (type Triangle) and as a
  one-triangle SceneMesh (type MeshTriangle, behind its exact Mesh.AABB gate,
  Scene.cs:67) — Möller–Trumbore, RMath.cs:29-73;
* AABB cases: a SceneMesh whose Mesh.AABB is the case's box and whose one
  triangle is a large plate across the ray inside the box, so the query hits
  exactly when the slab test (RMath.RayAABBIntersection, RMath.cs:12-26) of
  the gate passes.

Every answer is compared bitwise with the hand-derived value and with the
brute-force CPU oracle on the same scene."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))
BUILDS = [0, 1]  # RT_BUILD_SAH_HOST, RT_BUILD_LBVH_GPU

# ObjectType, ObjectType.cs:3-9
NONE, SPHERE, TRIANGLE, MESH_TRIANGLE = 0, 1, 2, 3


def _mat(rt):
    return rt.scene.MaterialData(DiffuseReflectance=(0.5, 0.5, 0.5))


def _query(gpu_ctx, orc, scene, ray, build):
    gpu_ctx.set_scene(scene, build)
    rays = np.asarray([ray], np.float32).reshape(1, 6)
    got = gpu_ctx.intersect_rays(rays)[0]
    ref = orc.intersect(scene, rays)[0]
    for f in ("type", "index", "mesh_index"):
        assert got[f] == ref[f], f
    assert np.float32(got["distance"]).view(np.uint32) == np.float32(ref["distance"]).view(np.uint32)
    return got


def _check_hit(got, case, want_type):
    if case["hit"]:
        assert got["type"] == want_type and got["index"] == 0
        assert np.float32(got["distance"]).view(np.uint32) == np.float32(case["t"]).view(np.uint32)
    else:
        assert got["type"] == NONE and got["index"] == -1
        assert got["distance"] == np.finfo(np.float32).max  # float.MaxValue, Scene.cs:45


@pytest.mark.parametrize("build", BUILDS)
@pytest.mark.parametrize("case", KAT["sphere"], ids=lambda c: c["name"])
def test_kat_sphere_gpu(rt, gpu_ctx, orc, case, build):
    S = rt.Scene()
    c = case["sphere"]
    S.add_sphere_r2(c[:3], c[3], _mat(rt))
    got = _query(gpu_ctx, orc, S, case["ray"], build)
    _check_hit(got, case, SPHERE)


@pytest.mark.parametrize("build", BUILDS)
@pytest.mark.parametrize("as_mesh", [False, True], ids=["loose", "mesh"])
@pytest.mark.parametrize("case", KAT["triangle"], ids=lambda c: c["name"])
def test_kat_triangle_gpu(rt, gpu_ctx, orc, case, as_mesh, build):
    tri = np.asarray(case["tri"], np.float32).reshape(1, 3, 3)
    S = rt.Scene()
    if as_mesh:
        S.add_mesh(rt.scene.Mesh.from_vertices(tri.reshape(3, 3), [0, 1, 2], _mat(rt)))
    else:
        S.add_triangles(tri, [_mat(rt)])
    got = _query(gpu_ctx, orc, S, case["ray"], build)
    _check_hit(got, case, MESH_TRIANGLE if as_mesh else TRIANGLE)
    if as_mesh and case["hit"]:
        assert got["mesh_index"] == 0


def _plate(ray):
    """A large triangle across the ray, 2.5 along its direction from the
    origin (inside every case box along the ray), perpendicular to it."""
    o = np.asarray(ray[:3], np.float64)
    d = np.asarray(ray[3:], np.float64)
    d = d / np.linalg.norm(d)
    p = o + 2.5 * d
    a = np.cross(d, [1.0, 0.0, 0.0] if abs(d[0]) < 0.9 else [0.0, 1.0, 0.0])
    a /= np.linalg.norm(a)
    b = np.cross(d, a)
    R = 40.0
    verts = [p + R * a, p + R * (-0.5 * a + 0.866 * b), p + R * (-0.5 * a - 0.866 * b)]
    return np.asarray(verts, np.float32)


@pytest.mark.parametrize("build", BUILDS)
@pytest.mark.parametrize("case", KAT["aabb"], ids=lambda c: c["name"])
def test_kat_aabb_gate_gpu(rt, gpu_ctx, orc, case, build):
    box = np.asarray(case["box"], np.float32).reshape(2, 3)
    plate = _plate(case["ray"])
    # the plate really crosses the ray inside the box (so a hit <=> the gate passes)
    hit_t = orc.ray_triangle(case["ray"], plate.reshape(-1).tolist())
    assert hit_t[0]
    m = rt.scene.Mesh.from_vertices(plate, [0, 1, 2], _mat(rt))
    m.AABB = box  # Mesh.AABB as the caller computed it: the case's box is the gate
    S = rt.Scene()
    S.add_mesh(m)
    got = _query(gpu_ctx, orc, S, case["ray"], build)
    assert (got["type"] == MESH_TRIANGLE) == case["hit"], case["name"]
    assert orc.ray_aabb(case["ray"], case["box"]) == case["hit"]
