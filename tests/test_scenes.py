"""Scene fixtures and the host-side extraction semantics (CPU only)."""
import numpy as np

f32 = np.float32


def test_config_sizes(rt):
    assert rt.make("C1").scene.triangle_count == 10
    assert rt.make("C2").scene.triangle_count == 32
    c3 = rt.make("C3")
    assert c3.scene.triangle_count == 69120 + 12
    assert (c3.plane.ResolutionX, c3.plane.ResolutionY, c3.spp, c3.max_bounces) == (1920, 1080, 4, 8)
    c5 = rt.make("C5")
    assert sum(len(m.Triangles) for m in c5.scene.Meshes) == 20833 * 12 == 249996
    assert (c5.spp, c5.max_bounces) == (64, 16)
    c4 = rt.make("C4")
    assert (c4.plane.ResolutionX, c4.plane.ResolutionY, c4.spp) == (3840, 2160, 16)


def test_deterministic(rt):
    a, b = rt.make("C5").scene, rt.make("C5").scene
    assert all(np.array_equal(x.Triangles, y.Triangles) for x, y in zip(a.Meshes, b.Meshes))


def test_normals_face_the_room(rt):
    """Loose room triangles shade with +Triangle.Normal (FetchTriangles,
    RayTracingSetup.cs:166); mesh triangles with -Triangle.Normal
    (SceneMesh.cs:43).  Fixtures are wound so both face the viewer side."""
    sc = rt.make("C2").scene
    tris = sc.TriangleData.Triangles
    cen = tris.mean(1)
    n = sc.TriangleData.Normals
    inward = -cen
    inward[:, 1] = np.where(np.abs(cen[:, 1]) > 0.98, -cen[:, 1], inward[:, 1])
    assert np.all((n * inward).sum(1) > 0)
    for m in sc.Meshes:
        box_c = m.Triangles.reshape(-1, 3).mean(0)
        out = m.Triangles.mean(1) - box_c
        assert np.all((m.TriangleNormals * out).sum(1) > 0)


def test_mesh_extraction_semantics(rt):
    """SceneMesh.Mesh: AABB over all transformed vertices, normals negated."""
    verts, idx = rt.scenes.unit_cube()
    m = rt.Mesh.from_vertices(verts, idx, rt.MaterialData())
    assert m.Triangles.shape == (12, 3, 3)
    assert np.array_equal(m.AABB, np.array([[-0.5] * 3, [0.5] * 3], f32))
    n = rt.scene.triangle_normal(m.Triangles)
    assert np.array_equal(m.TriangleNormals, -n)
    # outward: normal points away from the cube center
    assert np.all((m.TriangleNormals * m.Triangles.mean(1)).sum(1) > 0)


def test_trs_identity_exact(rt):
    m = rt.scene.quaternion_trs((0, 0, 0), (0, 0, 0, 1), (1, 1, 1))
    v = np.array([[1.5, -2.25, 3.125]], f32)
    assert np.array_equal(rt.scene.multiply_point3x4(m, v), v)


def test_scene_desc_roundtrip(rt, orc):
    fr = rt.make("demo")
    box = orc.scene_aabb(fr.scene)
    # Scene.CalculateAABB: sphere r = 10 around (0,0,29.6) is inside the bounds
    assert box[0, 2] <= 19.6 and box[1, 2] >= 39.6
    d = fr.scene.to_desc()
    assert d.desc.mesh_count == 1 and d.desc.triangle_count == 2 and d.desc.sphere_count == 1
