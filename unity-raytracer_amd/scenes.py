"""Scene fixtures for the configs of BASELINE.json and the reference demo.

The reference ships exactly one authored scene (Assets/RayTracer/Demo-RayTracing/
RayTracing.unity) and none of the BASELINE scenes, so the
configs are deterministic procedural stand-ins (seed 20250101), defined in
SURVEY.md §8(d):

  C1 cornell_c1   Cornell room, 10 wall tris + 2 spheres (1 mirror), 1 light, 256x256, 1 spp, depth 1
  C2 cornell_c2   room + light quad + short/tall box meshes = 32 tris, 3 spheres (2 mirror), 1080p, 4 spp, depth 8
  C3 knot_c3      room + light quad + (2,3) torus-knot tube mesh 384x90x2 = 69,120 tris + spheres, 1080p, 4 spp, depth 8
  C4 = C3 at 3840x2160, 16 spp, depth 8 (8 GPUs)
  C5 hall_c5      room + 20,833 random box meshes (249,996 tris, 10 % mirrors), 1080p, 64 spp, depth 16

Every fixture returns a ``Frame``: the Scene plus CameraData, ImagePlane and
RayTracingSetup's BackgroundColor / MaxReflectionBounces, i.e. everything
CastPixelRays reads (RayTracingSetup.cs:21-23,275-302).
"""
from __future__ import annotations

from dataclasses import dataclass, replace

import numpy as np

from .scene import MaterialData, Mesh, MeshSource, Scene, quaternion_trs, triangle_normal

f32 = np.float32
SEED = 20250101


@dataclass
class CameraData:
    """Data/Camera/CameraData.cs:5-11."""
    Position: tuple = (0.0, 0.0, 0.0)
    Forward: tuple = (0.0, 0.0, 1.0)
    Right: tuple = (1.0, 0.0, 0.0)
    Up: tuple = (0.0, 1.0, 0.0)


@dataclass
class ImagePlane:
    """Data/Camera/ImagePlane.cs:11-45 (Resolution inlined)."""
    ResolutionX: int = 50
    ResolutionY: int = 50
    DistanceToCamera: float = 10.0
    HalfHorizontalLength: float = 20.0
    HalfVerticalLength: float = 10.0


@dataclass
class Frame:
    name: str
    scene: Scene
    camera: CameraData
    plane: ImagePlane
    background: tuple = (0.0, 0.0, 0.0, 1.0)
    max_bounces: int = 0
    spp: int = 1

    def with_resolution(self, rx: int, ry: int) -> "Frame":
        return replace(self, plane=replace(self.plane, ResolutionX=rx, ResolutionY=ry))

    def with_(self, **kw) -> "Frame":
        return replace(self, **kw)


# ---------------------------------------------------------------------------
# The reference demo scene, RayTracing.unity (values cited per line)
# ---------------------------------------------------------------------------

def unit_cube():
    """A 24-vertex / 12-triangle unit cube on [-0.5, 0.5]^3 standing in for
    Unity's built-in Cube mesh (fileID 10202, Cube.prefab:44), whose vertex
    data is not in the reference.  Each face is wound so the mesh normal
    (-Triangle.Normal, SceneMesh.cs:43) points outward."""
    faces = [  # (normal axis, sign)
        (0, 1), (0, -1), (1, 1), (1, -1), (2, 1), (2, -1)]
    verts, idx = [], []
    for axis, sign in faces:
        u, v = [a for a in range(3) if a != axis]
        quad = []
        for (a, b) in ((-1, -1), (1, -1), (1, 1), (-1, 1)):
            p = [0.0, 0.0, 0.0]
            p[axis] = 0.5 * sign
            p[u] = 0.5 * a
            p[v] = 0.5 * b
            quad.append(p)
        base = len(verts)
        verts.extend(quad)
        tri_a = [base, base + 1, base + 2]
        tri_b = [base, base + 2, base + 3]
        # mesh normal = cross(v1 - v0, v2 - v0) direction; flip to outward
        p0, p1, p2 = (np.array(quad[i]) for i in (0, 1, 2))
        n = np.cross(p1 - p0, p2 - p0)
        if n[axis] * sign < 0:
            tri_a = [tri_a[0], tri_a[2], tri_a[1]]
            tri_b = [tri_b[0], tri_b[2], tri_b[1]]
        idx.extend(tri_a + tri_b)
    return np.array(verts, f32), np.array(idx, np.int32)


def demo_cube_source() -> MeshSource:
    """The demo's Cube before extraction (RayTracing.unity:395-422)."""
    cube_mat = MaterialData(DiffuseReflectance=(0, 1, 1))                               # Cube.prefab:100-118
    verts, idx = unit_cube()
    l2w = quaternion_trs((-24.7, 1.5497656e-6, 27.6),
                         (-0.37513673, 0.13105033, 0.3026398, 0.8663183),
                         (28.664, 10, 10))                                              # :395-422, Cube.prefab:31
    return MeshSource(verts, idx, l2w, cube_mat)


def without_meshes(sc: Scene) -> Scene:
    """The non-mesh part of a scene (the base of rt_set_scene_source)."""
    return Scene(TriangleData=sc.TriangleData, Meshes=[], SphereData=sc.SphereData,
                 PointLights=sc.PointLights, AmbientLight=sc.AmbientLight)


def demo_scene() -> Frame:
    """Assets/RayTracer/Demo-RayTracing/RayTracing.unity with prefab defaults.

    Renderer (:346-364): 50x50, DistanceToCamera 10, half 20 x 10, black
    background, MaxReflectionBounces 5.  Main Camera (:196-205) at the origin,
    identity rotation.  Object order (FindObjectsOfType order is unspecified
    in Unity) is fixed here: Triangle, Triangle (1); Sphere; Cube; PointLight.
    """
    sc = Scene()
    tri_mat = MaterialData(DiffuseReflectance=(0, 1, 0), AmbientReflectance=(1, 1, 1))  # Triangle.prefab:59-67
    tri_mat1 = MaterialData(DiffuseReflectance=(1, 0, 1), AmbientReflectance=(1, 1, 1))  # RayTracing.unity:251-262
    offs = ((0, 10, 0), (-10, -10, 0), (10, -10, 0))                                   # Triangle.prefab:47-58
    sc.add_triangle((17.1, 0, 15), *offs, tri_mat)                                      # RayTracing.unity:586-597
    sc.add_triangle((14.16, 0, 21.45), *offs, tri_mat1)                                 # RayTracing.unity:275-286
    # Sphere.prefab:99-117 with IsMirror / Specular overridden to 0 (RayTracing.unity:444-459)
    sph_mat = MaterialData(DiffuseReflectance=(1, 0, 0), AmbientReflectance=(1, 1, 1),
                           MirrorReflectance=(1, 1, 1), SpecularReflectance=(0, 0, 0),
                           PhongExponent=20, IsMirror=False)
    sc.add_sphere((0, 0, 29.6), 20.0, sph_mat)                                          # :472-475, Sphere.prefab:31
    sc.add_mesh(demo_cube_source().extract())
    sc.add_point_light((5.79, 0, 0), 100000.0)                                          # :643-654, PointLight.prefab:47
    sc.AmbientLight = np.array([15, 15, 15], f32)                                       # AmbientLight.prefab:47-51
    return Frame("demo", sc, CameraData(), ImagePlane(50, 50, 10.0, 20.0, 10.0),
                 background=(0.0, 0.0, 0.0, 1.0), max_bounces=5, spp=1)


# ---------------------------------------------------------------------------
# Cornell-style room used by C1-C5
# ---------------------------------------------------------------------------

WHITE = MaterialData(DiffuseReflectance=(0.75, 0.75, 0.75), AmbientReflectance=(0.1, 0.1, 0.1))
RED = MaterialData(DiffuseReflectance=(0.75, 0.12, 0.1), AmbientReflectance=(0.1, 0.02, 0.02))
GREEN = MaterialData(DiffuseReflectance=(0.12, 0.7, 0.15), AmbientReflectance=(0.02, 0.1, 0.02))
LAMP = MaterialData(DiffuseReflectance=(1, 1, 1), AmbientReflectance=(1.0, 1.0, 0.9))
MIRROR = MaterialData(DiffuseReflectance=(0.02, 0.02, 0.02), AmbientReflectance=(0.0, 0.0, 0.0),
                      MirrorReflectance=(0.8, 0.8, 0.8), SpecularReflectance=(0.6, 0.6, 0.6),
                      PhongExponent=64.0, IsMirror=True)
BLUE_PLASTIC = MaterialData(DiffuseReflectance=(0.15, 0.3, 0.8), AmbientReflectance=(0.02, 0.04, 0.1),
                            SpecularReflectance=(0.5, 0.5, 0.5), PhongExponent=32.0)
BOX_MAT = MaterialData(DiffuseReflectance=(0.7, 0.7, 0.62), AmbientReflectance=(0.08, 0.08, 0.07),
                       SpecularReflectance=(0.1, 0.1, 0.1), PhongExponent=8.0)
KNOT_MAT = MaterialData(DiffuseReflectance=(0.8, 0.55, 0.15), AmbientReflectance=(0.1, 0.07, 0.02),
                        SpecularReflectance=(0.4, 0.4, 0.4), PhongExponent=24.0)

LIGHT_POS = (0.0, 0.95, 0.0)
LIGHT_I = 600.0
AMBIENT = (25.0, 25.0, 25.0)


def _oriented_quad(a, b, c, d, inward_point, mat, out_tris, out_mats, loose=True):
    """Two triangles (a,b,c), (a,c,d) wound so the shading normal faces
    inward_point: loose triangles shade with +Triangle.Normal, meshes with
    -Triangle.Normal."""
    tris = np.array([[a, b, c], [a, c, d]], f32)
    n = triangle_normal(tris)
    if not loose:
        n = -n
    center = tris.reshape(-1, 3).mean(0)
    if np.dot(n[0], np.asarray(inward_point, f32) - center) < 0:
        tris = tris[:, [0, 2, 1]]
    out_tris.append(tris)
    out_mats.extend([mat, mat])


def add_room(sc: Scene, with_lamp: bool):
    """Room [-1,1]^3 open at -z: floor, ceiling, back, left (red), right
    (green) as 10 loose triangles (SceneTriangle); optional 2-triangle lamp
    quad just under the ceiling."""
    tris, mats = [], []
    c = (0.0, 0.0, 0.0)
    _oriented_quad((-1, -1, -1), (1, -1, -1), (1, -1, 1), (-1, -1, 1), c, WHITE, tris, mats)   # floor
    _oriented_quad((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1), c, WHITE, tris, mats)       # ceiling
    _oriented_quad((-1, -1, 1), (1, -1, 1), (1, 1, 1), (-1, 1, 1), c, WHITE, tris, mats)       # back
    _oriented_quad((-1, -1, -1), (-1, -1, 1), (-1, 1, 1), (-1, 1, -1), c, RED, tris, mats)     # left
    _oriented_quad((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1), c, GREEN, tris, mats)       # right
    if with_lamp:
        y = 0.99
        _oriented_quad((-0.25, y, -0.25), (0.25, y, -0.25), (0.25, y, 0.25), (-0.25, y, 0.25),
                       (0, -1, 0), LAMP, tris, mats)
    sc.add_triangles(np.concatenate(tris), mats)


def box_mesh_tris(center, size, yaw, with_bottom=True):
    """World-space triangles of a yawed box, wound for outward mesh normals."""
    hx, hy, hz = (0.5 * s for s in size)
    cy, sy = np.cos(yaw), np.sin(yaw)
    corners = []
    for dx, dy, dz in [(-1, -1, -1), (1, -1, -1), (1, -1, 1), (-1, -1, 1),
                       (-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)]:
        x, y, z = dx * hx, dy * hy, dz * hz
        corners.append((center[0] + cy * x + sy * z, center[1] + y, center[2] - sy * x + cy * z))
    corners = np.array(corners, np.float64)
    faces = [(4, 5, 6, 7), (0, 1, 5, 4), (1, 2, 6, 5), (2, 3, 7, 6), (3, 0, 4, 7)]
    if with_bottom:
        faces.append((0, 1, 2, 3))
    tris, mats = [], []
    for f in faces:
        _oriented_quad(*(corners[i] for i in f), center, None, tris, mats, loose=False)
        # _oriented_quad orients toward `center` (inward); flip to outward
        tris[-1] = tris[-1][:, [0, 2, 1]]
    return np.concatenate(tris).astype(f32), corners.astype(f32)


def _mesh_from_tris(tris, corners, mat) -> Mesh:
    verts = tris.reshape(-1, 3)
    idx = np.arange(len(verts), dtype=np.int32)
    m = Mesh.from_vertices(verts, idx, mat)
    # Mesh.AABB covers ALL vertices of the mesh (SceneMesh.cs:26-31): the
    # corner set equals the triangle vertex set here.
    return m


def _camera_room():
    return CameraData(Position=(0.0, 0.0, -3.4))


def cornell_c1() -> Frame:
    """C1: room + 2 spheres (one mirror) + 1 light, 256x256, 1 spp, depth 1."""
    sc = Scene()
    add_room(sc, with_lamp=False)
    sc.add_sphere_r2((-0.45, -0.6, 0.35), 0.4 * 0.4, MIRROR)
    sc.add_sphere_r2((0.5, -0.65, -0.2), 0.35 * 0.35, BLUE_PLASTIC)
    sc.add_point_light(LIGHT_POS, LIGHT_I)
    sc.AmbientLight = np.array(AMBIENT, f32)
    return Frame("C1", sc, _camera_room(), ImagePlane(256, 256, 1.0, 0.5, 0.5),
                 background=(0.0, 0.0, 0.0, 1.0), max_bounces=1, spp=1)


def _c2_scene(with_boxes=True) -> Scene:
    sc = Scene()
    if with_boxes:
        t, c = box_mesh_tris((0.4, -0.7, -0.25), (0.55, 0.6, 0.55), 0.3, with_bottom=False)
        sc.add_mesh(_mesh_from_tris(t, c, BOX_MAT))
        t, c = box_mesh_tris((-0.4, -0.4, 0.35), (0.55, 1.2, 0.55), -0.28, with_bottom=False)
        sc.add_mesh(_mesh_from_tris(t, c, BOX_MAT))
    add_room(sc, with_lamp=True)
    return sc


def cornell_c2() -> Frame:
    """C2: room + lamp quad + short/tall boxes (32 tris) + 3 spheres (2 mirror),
    1920x1080, 4 spp, depth 8."""
    sc = _c2_scene()
    sc.add_sphere_r2((0.4, -0.1, -0.25), 0.3 * 0.3, MIRROR)
    sc.add_sphere_r2((-0.4, 0.5, 0.35), 0.3 * 0.3, MIRROR)
    sc.add_sphere_r2((0.55, -0.75, -0.75), 0.2 * 0.2, BLUE_PLASTIC)
    sc.add_point_light(LIGHT_POS, LIGHT_I)
    sc.AmbientLight = np.array(AMBIENT, f32)
    assert sc.triangle_count == 32
    return Frame("C2", sc, _camera_room(), ImagePlane(1920, 1080, 1.0, 0.8889, 0.5),
                 background=(0.0, 0.0, 0.0, 1.0), max_bounces=8, spp=4)


def mirror_corridor(depth=40, res=(24, 12), spp=1, loose=True) -> Frame:
    """Two facing mirror walls (x = -1, x = +1; km 0.9, 0.8, 0.7) along a
    400-unit corridor with a white floor, a mirror sphere, a point light and an
    ambient light; the camera looks down the corridor through a wide image
    plane, so rays bounce between the walls tens of times — mirror chains
    deeper than the library's 32-entry fold stack (MaxReflectionBounces is an
    unbounded int in the reference, RayTracingSetup.cs:23,358).  loose=False:
    the walls as one mesh (SceneMesh) instead of loose triangles."""
    wall = MaterialData(DiffuseReflectance=(0.2, 0.2, 0.2), AmbientReflectance=(0.05, 0.05, 0.05),
                        MirrorReflectance=(0.9, 0.8, 0.7), SpecularReflectance=(0.3, 0.3, 0.3),
                        PhongExponent=16.0, IsMirror=True)
    sc = Scene()
    tris, mats = [], []
    L = 200.0
    _oriented_quad((-1, -1, -L), (-1, -1, L), (-1, 1, L), (-1, 1, -L), (0, 0, 0), wall, tris, mats, loose)
    _oriented_quad((1, -1, -L), (1, -1, L), (1, 1, L), (1, 1, -L), (0, 0, 0), wall, tris, mats, loose)
    _oriented_quad((-1, -1, -L), (1, -1, -L), (1, -1, L), (-1, -1, L), (0, 0, 0), WHITE, tris, mats, True)
    t = np.concatenate(tris)
    if loose:
        sc.add_triangles(t, mats)
    else:
        sc.add_mesh(_mesh_from_tris(t[:4], t[:4].reshape(-1, 3), wall))
        sc.add_triangles(t[4:], mats[4:])
    sc.add_sphere_r2((0.3, -0.5, 12.0), 0.25, MIRROR)
    sc.add_point_light((0.0, 0.9, 4.0), 300.0)
    sc.AmbientLight = np.array(AMBIENT, f32)
    cam = CameraData(Position=(0.1, 0.05, -3.4))
    return Frame(f"corridor{depth}", sc, cam, ImagePlane(res[0], res[1], 1.0, 2.5, 0.08),
                 background=(0.1, 0.2, 0.3, 1.0), max_bounces=depth, spp=spp)


def torus_knot(p=2, q=3, segments=384, sides=90, scale=0.22, tube=0.085, center=(0.0, -0.15, 0.15)):
    """(p,q) torus-knot tube: segments x sides quads = 2*segments*sides tris."""
    phi = np.arange(segments, dtype=np.float64) * (2 * np.pi / segments)

    def curve(t):
        r = 2.0 + np.cos(q * t)
        return np.stack([r * np.cos(p * t), r * np.sin(p * t), np.sin(q * t)], -1) * scale

    c = curve(phi)
    eps = 1e-4
    tang = curve(phi + eps) - curve(phi - eps)
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    acc = curve(phi + eps) - 2 * c + curve(phi - eps)
    nrm = acc - (acc * tang).sum(1, keepdims=True) * tang
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    bin_ = np.cross(tang, nrm)
    theta = np.arange(sides, dtype=np.float64) * (2 * np.pi / sides)
    ring = (np.cos(theta)[None, :, None] * nrm[:, None, :] + np.sin(theta)[None, :, None] * bin_[:, None, :])
    verts = (c[:, None, :] + tube * ring + np.asarray(center)[None, None, :]).reshape(-1, 3)
    i = np.arange(segments)[:, None]
    j = np.arange(sides)[None, :]
    a = i * sides + j
    b = ((i + 1) % segments) * sides + j
    c2 = ((i + 1) % segments) * sides + (j + 1) % sides
    d = i * sides + (j + 1) % sides
    idx = np.stack([np.stack([a, b, c2], -1), np.stack([a, c2, d], -1)], 2).reshape(-1, 3)
    # orient for outward mesh normals: cross(v1 - v0, v2 - v0) along ring dir
    v0, v1, v2 = verts[idx[0, 0]], verts[idx[0, 1]], verts[idx[0, 2]]
    out = np.cross(v1 - v0, v2 - v0)
    if np.dot(out, ring[0, 0]) < 0:
        idx = idx[:, [0, 2, 1]]
    return verts.astype(f32), idx.astype(np.int32)


def knot_c3() -> Frame:
    """C3: room + lamp + 69,120-triangle torus-knot mesh (stand-in for the
    ~69k-triangle Stanford Bunny, not available offline) + mirror and diffuse
    spheres; 1920x1080, 4 spp, depth 8."""
    sc = Scene()
    verts, idx = torus_knot()
    sc.add_mesh(Mesh.from_vertices(verts, idx, KNOT_MAT))
    add_room(sc, with_lamp=True)
    sc.add_sphere_r2((-0.62, -0.68, -0.45), 0.3 * 0.3, MIRROR)
    sc.add_sphere_r2((0.65, -0.75, -0.55), 0.25 * 0.25, BLUE_PLASTIC)
    sc.add_point_light(LIGHT_POS, LIGHT_I)
    sc.AmbientLight = np.array(AMBIENT, f32)
    assert sc.triangle_count == 69120 + 12
    return Frame("C3", sc, _camera_room(), ImagePlane(1920, 1080, 1.0, 0.8889, 0.5),
                 background=(0.0, 0.0, 0.0, 1.0), max_bounces=8, spp=4)


def knot_c4() -> Frame:
    """C4: C3 at 3840x2160, 16 spp, depth 8."""
    return knot_c3().with_(name="C4", spp=16).with_resolution(3840, 2160)


def hall_c5(n_boxes=20833, seed=SEED) -> Frame:
    """C5: room + n_boxes seeded random yawed boxes, one SceneMesh each
    (12 tris; sizes U[0.02,0.2], positions U over the room, yaw U[0,2pi),
    10 % mirrors) = 249,996 box triangles; 1920x1080, 64 spp, depth 16."""
    rng = np.random.default_rng(seed)
    sc = Scene()
    sizes = rng.uniform(0.02, 0.2, (n_boxes, 3))
    pos = rng.uniform(-0.9, 0.9, (n_boxes, 3))
    yaw = rng.uniform(0.0, 2 * np.pi, n_boxes)
    mirror = rng.uniform(0.0, 1.0, n_boxes) < 0.1
    # keep the point light outside every box
    far = np.linalg.norm(pos - np.asarray(LIGHT_POS), axis=1) > 0.25
    tris_all, meshes = _boxes_vectorized(pos, sizes, yaw)
    for k in range(n_boxes):
        if not far[k]:
            # move the box below the light instead of dropping it (keeps the count)
            pos[k, 1] = -0.5
    tris_all, _ = _boxes_vectorized(pos, sizes, yaw)
    mmat = MIRROR
    for k in range(n_boxes):
        t = tris_all[k]
        aabb = np.stack([t.reshape(-1, 3).min(0), t.reshape(-1, 3).max(0)]).astype(f32)
        normals = (-triangle_normal(t)).astype(f32)
        sc.Meshes.append(Mesh(t, normals, mmat if mirror[k] else BOX_MAT, aabb))
    add_room(sc, with_lamp=True)
    sc.add_point_light(LIGHT_POS, LIGHT_I)
    sc.AmbientLight = np.array(AMBIENT, f32)
    return Frame("C5", sc, _camera_room(), ImagePlane(1920, 1080, 1.0, 0.8889, 0.5),
                 background=(0.0, 0.0, 0.0, 1.0), max_bounces=16, spp=64)


def yaw_quaternion(yaw):
    """Quaternion.Euler(0, yaw, 0) as (x, y, z, w) float32."""
    h = np.asarray(yaw, np.float64) * 0.5
    z = np.zeros_like(h)
    return np.stack([z, np.sin(h), z, np.cos(h)], -1).astype(f32)


def instanced_hall(n_boxes=20833, seed=SEED, res=(1920, 1080), spp=4, bounces=8):
    """Animated variant of C5 for device-side extraction: n_boxes instances of
    the unit cube, each a SceneMesh with its own Transform (position, yaw,
    scale), inside the C2 room.  Returns (Frame with an empty-mesh base scene,
    [MeshSource], matrices(t) -> (n, 4, 4)).  At time t every box spins about
    y and bobs vertically, so every frame needs re-extraction and a rebuild
    (UpdateScene, RayTracingSetup.cs:120-128)."""
    rng = np.random.default_rng(seed)
    sizes = rng.uniform(0.02, 0.2, (n_boxes, 3)).astype(f32)
    pos = rng.uniform(-0.9, 0.9, (n_boxes, 3)).astype(f32)
    yaw0 = rng.uniform(0.0, 2 * np.pi, n_boxes)
    spin = rng.uniform(-2.0, 2.0, n_boxes)
    phase = rng.uniform(0.0, 2 * np.pi, n_boxes)
    mirror = rng.uniform(0.0, 1.0, n_boxes) < 0.1
    near = np.linalg.norm(pos - np.asarray(LIGHT_POS, f32), axis=1) <= 0.35
    pos[near, 1] = -0.5
    verts, idx = unit_cube()

    def matrices(t: float) -> np.ndarray:
        q = yaw_quaternion(yaw0 + spin * t)
        p = pos.copy()
        p[:, 1] = (p[:, 1] + (0.05 * np.sin(phase + 3.0 * t))).astype(f32)
        return np.stack([quaternion_trs(p[k], q[k], sizes[k]) for k in range(n_boxes)])

    m0 = matrices(0.0)
    sources = [MeshSource(verts, idx, m0[k], MIRROR if mirror[k] else BOX_MAT) for k in range(n_boxes)]
    base = Scene()
    add_room(base, with_lamp=True)
    base.add_point_light(LIGHT_POS, LIGHT_I)
    base.AmbientLight = np.array(AMBIENT, f32)
    fr = Frame("C5i", base, _camera_room(), ImagePlane(res[0], res[1], 1.0, 0.8889, 0.5),
               background=(0.0, 0.0, 0.0, 1.0), max_bounces=bounces, spp=spp)
    return fr, sources, matrices


def extracted(fr: Frame, sources, mats=None) -> Frame:
    """Host extraction (SceneMesh.Mesh restated in scene.py) of `sources`
    with optional replacement matrices: the reference-side scene."""
    sc = Scene(TriangleData=fr.scene.TriangleData, Meshes=[], SphereData=fr.scene.SphereData,
               PointLights=fr.scene.PointLights, AmbientLight=fr.scene.AmbientLight)
    for k, src in enumerate(sources):
        m = src.LocalToWorld if mats is None else mats[k]
        sc.Meshes.append(Mesh.from_vertices(src.Vertices, src.Indices, src.MaterialData, m))
    return fr.with_(scene=sc)


def _boxes_vectorized(pos, sizes, yaw):
    """(n, 12, 3, 3) f32 triangles of n yawed boxes, outward mesh winding."""
    n = len(pos)
    sgn = np.array([(-1, -1, -1), (1, -1, -1), (1, -1, 1), (-1, -1, 1),
                    (-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)], np.float64)
    loc = sgn[None] * (0.5 * sizes)[:, None, :]
    cy, sy = np.cos(yaw)[:, None], np.sin(yaw)[:, None]
    wx = pos[:, 0:1] + cy * loc[..., 0] + sy * loc[..., 2]
    wy = pos[:, 1:2] + loc[..., 1]
    wz = pos[:, 2:3] - sy * loc[..., 0] + cy * loc[..., 2]
    corners = np.stack([wx, wy, wz], -1).astype(f32)          # (n, 8, 3)
    # faces with outward winding for cross(v1-v0, v2-v0) (right-handed axes)
    quads = [(4, 7, 6, 5), (0, 1, 2, 3), (0, 4, 5, 1), (1, 5, 6, 2), (2, 6, 7, 3), (3, 7, 4, 0)]
    tri_idx = []
    for a, b, c, d in quads:
        tri_idx += [(a, b, c), (a, c, d)]
    tri_idx = np.array(tri_idx)
    tris = corners[:, tri_idx]                                 # (n, 12, 3, 3)
    return tris, corners


CONFIGS = {
    "demo": demo_scene,
    "C1": cornell_c1,
    "C2": cornell_c2,
    "C3": knot_c3,
    "C4": knot_c4,
    "C5": hall_c5,
}


def make(name: str) -> Frame:
    return CONFIGS[name]()
