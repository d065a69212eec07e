"""Host-side mirror of the reference's scene data (Assets/RayTracer/Data/**)
and of its scene-extraction semantics (Assets/RayTracer/SceneComponents/*.cs).

Names follow the reference: ``Scene`` holds ``TriangleData``, ``MeshData``,
``SphereData``, ``PointLights`` and ``AmbientLight`` (Data/Objects/Scene.cs:8-13).
Geometry is kept as float32 numpy arrays so a scene of 250k triangles costs
nothing to build; every derived quantity (triangle normals, mesh AABBs,
world-space vertices, sphere radii) is computed with the reference's float32
operation order, so the bytes handed to the C-ABI are the bytes the Unity
side would hand over.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import abi

f32 = np.float32

MATERIAL_DTYPE = np.dtype([
    ("DiffuseReflectance", f32, 3),
    ("AmbientReflectance", f32, 3),
    ("MirrorReflectance", f32, 3),
    ("SpecularReflectance", f32, 3),
    ("PhongExponent", f32),
    ("IsMirror", np.int32),
], align=False)
assert MATERIAL_DTYPE.itemsize == C.sizeof(abi.rt_material) == 56

MESH_DTYPE = np.dtype([
    ("first_triangle", np.int32),
    ("triangle_count", np.int32),
    ("material", MATERIAL_DTYPE),
    ("aabb", f32, (2, 3)),
])
assert MESH_DTYPE.itemsize == C.sizeof(abi.rt_mesh) == 88


@dataclass
class MaterialData:
    """Data/Shading/MaterialData.cs:7-15."""
    DiffuseReflectance: tuple = (0.0, 0.0, 0.0)
    AmbientReflectance: tuple = (0.0, 0.0, 0.0)
    MirrorReflectance: tuple = (0.0, 0.0, 0.0)
    SpecularReflectance: tuple = (0.0, 0.0, 0.0)
    PhongExponent: float = 0.0
    IsMirror: bool = False

    def record(self):
        r = np.zeros((), MATERIAL_DTYPE)
        r["DiffuseReflectance"] = self.DiffuseReflectance
        r["AmbientReflectance"] = self.AmbientReflectance
        r["MirrorReflectance"] = self.MirrorReflectance
        r["SpecularReflectance"] = self.SpecularReflectance
        r["PhongExponent"] = self.PhongExponent
        r["IsMirror"] = 1 if self.IsMirror else 0
        return r


def materials_array(mats: List[MaterialData]) -> np.ndarray:
    out = np.zeros(len(mats), MATERIAL_DTYPE)
    for i, m in enumerate(mats):
        out[i] = m.record()
    return out


# ---------------------------------------------------------------------------
# Unity.Mathematics semantics used by scene extraction (float32, op order)
# ---------------------------------------------------------------------------

def _cross(a, b):
    """cross(x, y) = (x * y.yzx - x.yzx * y).yzx, per component a*b - c*d."""
    return np.stack([
        a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
        a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
        a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0],
    ], axis=-1)


def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _umin(x, y):
    """math.min(x, y) = isnan(y) || x < y ? x : y."""
    return np.where(np.isnan(y) | (x < y), x, y)


def _umax(x, y):
    return np.where(np.isnan(y) | (x > y), x, y)


def triangle_normal(tris: np.ndarray) -> np.ndarray:
    """Triangle.Normal (Data/Objects/Triangle.cs:13-21): v / length(v) with
    v = cross(Vertex2 - Vertex0, Vertex1 - Vertex0); tris is (N, 3, 3) f32."""
    tris = np.asarray(tris, f32)
    v = _cross(tris[:, 2] - tris[:, 0], tris[:, 1] - tris[:, 0])
    ln = np.sqrt(_dot(v, v))
    return (v / ln[:, None]).astype(f32)


def aabb_of_points(points: np.ndarray) -> np.ndarray:
    """AABB init Min=float.MaxValue, Max=float.MinValue then Encapsulate(point)
    for every point in order (SceneMesh.cs:22-31, AABB.cs:10-14)."""
    mn = np.full(3, np.finfo(f32).max, f32)
    mx = np.full(3, -np.finfo(f32).max, f32)
    pts = np.asarray(points, f32).reshape(-1, 3)
    if len(pts) == 0:
        return np.stack([mn, mx])
    # Encapsulate is an order-dependent fold only through NaN / signed zero;
    # min over finite float32 is order independent except -0 vs +0, which
    # never changes a later comparison.  Use the exact fold for small sets.
    if len(pts) <= 4096 or np.isnan(pts).any():
        for p in pts:
            mn = _umin(p, mn).astype(f32)
            mx = _umax(p, mx).astype(f32)
        return np.stack([mn, mx])
    return np.stack([np.minimum(mn, pts.min(0)), np.maximum(mx, pts.max(0))]).astype(f32)


def quaternion_trs(position, rotation_xyzw, scale) -> np.ndarray:
    """Matrix4x4.TRS(pos, rot, scale) (UnityEngine, closed source) restated in
    float32: R from the quaternion (Matrix4x4.Rotate), columns scaled by s,
    translation in the last column.  Unity computes localToWorldMatrix natively;
    this restatement is documented as parity-unpinned."""
    qx, qy, qz, qw = (f32(v) for v in rotation_xyzw)
    x, y, z = qx * f32(2), qy * f32(2), qz * f32(2)
    xx, yy, zz = qx * x, qy * y, qz * z
    xy, xz, yz = qx * y, qx * z, qy * z
    wx, wy, wz = qw * x, qw * y, qw * z
    one = f32(1)
    r = np.array([
        [one - (yy + zz), xy - wz, xz + wy],
        [xy + wz, one - (xx + zz), yz - wx],
        [xz - wy, yz + wx, one - (xx + yy)],
    ], f32)
    s = np.asarray(scale, f32)
    m = np.zeros((4, 4), f32)
    m[:3, :3] = r * s[None, :]
    m[:3, 3] = np.asarray(position, f32)
    m[3, 3] = one
    return m


def multiply_point3x4(m: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Matrix4x4.MultiplyPoint3x4: m00*x + m01*y + m02*z + m03 (left to right)."""
    v = np.asarray(v, f32)
    out = np.empty_like(v)
    for r in range(3):
        out[:, r] = ((m[r, 0] * v[:, 0] + m[r, 1] * v[:, 1]) + m[r, 2] * v[:, 2]) + m[r, 3]
    return out


@dataclass
class Mesh:
    """Data/Objects/Mesh.cs:7-13."""
    Triangles: np.ndarray          # (N, 3, 3) f32 world space
    TriangleNormals: np.ndarray    # (N, 3) f32 == -Triangle.Normal
    MaterialData: MaterialData
    AABB: np.ndarray               # (2, 3) f32 over ALL transformed vertices

    @staticmethod
    def from_vertices(vertices, indices, material: MaterialData, local_to_world=None) -> "Mesh":
        """SceneMesh.Mesh getter (SceneComponents/SceneMesh.cs:11-53): transform
        every vertex, AABB over all of them, triangles from the index buffer in
        order, normals = -Triangle.Normal."""
        verts = np.asarray(vertices, f32).reshape(-1, 3)
        if local_to_world is not None:
            verts = multiply_point3x4(local_to_world, verts)
        aabb = aabb_of_points(verts)
        idx = np.asarray(indices, np.int64).reshape(-1, 3)
        tris = verts[idx]
        normals = (-triangle_normal(tris)).astype(f32)
        return Mesh(tris.astype(f32), normals, material, aabb)


@dataclass
class MeshSource:
    """A SceneMesh before extraction (SceneComponents/SceneMesh.cs:11-53):
    MeshFilter.sharedMesh (local vertices + index buffer), the transform's
    localToWorldMatrix and the MaterialData.  ``extract()`` is the host
    restatement of the SceneMesh.Mesh getter; rt_set_scene_source runs the
    same extraction on the device."""
    Vertices: np.ndarray       # (V, 3) f32 local space
    Indices: np.ndarray        # (3T,) int32
    LocalToWorld: np.ndarray   # (4, 4) f32, row-major
    MaterialData: MaterialData

    def extract(self) -> "Mesh":
        return Mesh.from_vertices(self.Vertices, self.Indices, self.MaterialData, self.LocalToWorld)


class MeshSourceArray:
    """ctypes rt_mesh_source[] over contiguous numpy arrays (kept alive here)."""

    def __init__(self, sources: List[MeshSource]):
        self.keep = []
        self.arr = (abi.rt_mesh_source * max(1, len(sources)))()
        self.count = len(sources)
        for i, src in enumerate(sources):
            v = np.ascontiguousarray(src.Vertices, f32).reshape(-1, 3)
            ix = np.ascontiguousarray(src.Indices, np.int32).reshape(-1)
            self.keep += [v, ix]
            e = self.arr[i]
            e.vertices = v.ctypes.data if v.size else None
            e.vertex_count = len(v)
            e.indices = ix.ctypes.data if ix.size else None
            e.index_count = len(ix)
            e.local_to_world[:] = [float(x) for x in np.asarray(src.LocalToWorld, f32).reshape(16)]
            e.material = abi.rt_material.from_buffer_copy(src.MaterialData.record().tobytes())

    def ptr(self):
        return C.cast(self.arr, C.c_void_p)


@dataclass
class TriangleData:
    """Data/Objects/TriangleData.cs:8-13."""
    Triangles: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 3), f32))
    Normals: np.ndarray = field(default_factory=lambda: np.zeros((0, 3), f32))
    Materials: List[MaterialData] = field(default_factory=list)


@dataclass
class SphereData:
    """Data/Objects/SphereData.cs:7-10; Spheres rows = (Center.xyz, RadiusSquared)."""
    Spheres: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), f32))
    Materials: List[MaterialData] = field(default_factory=list)


@dataclass
class Scene:
    """Data/Objects/Scene.cs:6-15 (AABB is computed by the library,
    Scene.CalculateAABB, on rt_set_scene)."""
    TriangleData: TriangleData = field(default_factory=TriangleData)
    Meshes: List[Mesh] = field(default_factory=list)            # MeshData.Meshes
    SphereData: SphereData = field(default_factory=SphereData)
    PointLights: np.ndarray = field(default_factory=lambda: np.zeros((0, 6), f32))  # (pos, intensity)
    AmbientLight: np.ndarray = field(default_factory=lambda: np.zeros(3, f32))      # Radiance

    # ---- extraction helpers (SceneComponents/*.cs) ----
    def add_triangle(self, position, offset0, offset1, offset2, material: MaterialData):
        """SceneTriangle (SceneTriangle.cs:16-22) + FetchTriangles (:159-169)."""
        c = np.asarray(position, f32)
        tri = np.stack([c + np.asarray(offset0, f32), c + np.asarray(offset1, f32),
                        c + np.asarray(offset2, f32)])[None]
        self.add_triangles(tri, [material])

    def add_triangles(self, tris, materials: List[MaterialData]):
        tris = np.asarray(tris, f32).reshape(-1, 3, 3)
        assert len(materials) == len(tris)
        td = self.TriangleData
        td.Triangles = np.concatenate([td.Triangles, tris])
        td.Normals = np.concatenate([td.Normals, triangle_normal(tris)])
        td.Materials = td.Materials + list(materials)

    def add_sphere(self, position, scale_x: float, material: MaterialData):
        """SceneSphere.Sphere (SceneSphere.cs:9-22): radius = scale.x * 0.5f."""
        radius = f32(scale_x) * f32(0.5)
        row = np.array([[*np.asarray(position, f32), radius * radius]], f32)
        self.SphereData.Spheres = np.concatenate([self.SphereData.Spheres, row])
        self.SphereData.Materials = self.SphereData.Materials + [material]

    def add_sphere_r2(self, center, radius_squared: float, material: MaterialData):
        row = np.array([[*np.asarray(center, f32), f32(radius_squared)]], f32)
        self.SphereData.Spheres = np.concatenate([self.SphereData.Spheres, row])
        self.SphereData.Materials = self.SphereData.Materials + [material]

    def add_point_light(self, position, intensity: float):
        """ScenePointLight.Light (ScenePointLight.cs:9-13): float → float3."""
        i = f32(intensity)
        row = np.array([[*np.asarray(position, f32), i, i, i]], f32)
        self.PointLights = np.concatenate([self.PointLights, row])

    def add_mesh(self, mesh: Mesh):
        self.Meshes.append(mesh)

    # ---- statistics ----
    @property
    def triangle_count(self) -> int:
        return len(self.TriangleData.Triangles) + sum(len(m.Triangles) for m in self.Meshes)

    # ---- C-ABI descriptor ----
    def to_desc(self) -> "SceneDesc":
        return SceneDesc(self)


class SceneDesc:
    """rt_scene_desc backed by contiguous numpy arrays (kept alive here)."""

    def __init__(self, scene: Scene):
        td = scene.TriangleData
        self.triangles = np.ascontiguousarray(td.Triangles, f32).reshape(-1, 9)
        self.triangle_normals = np.ascontiguousarray(td.Normals, f32).reshape(-1, 3)
        self.triangle_materials = materials_array(td.Materials)
        if scene.Meshes:
            self.mesh_triangles = np.ascontiguousarray(
                np.concatenate([m.Triangles.reshape(-1, 9) for m in scene.Meshes]), f32)
            self.mesh_normals = np.ascontiguousarray(
                np.concatenate([m.TriangleNormals.reshape(-1, 3) for m in scene.Meshes]), f32)
        else:
            self.mesh_triangles = np.zeros((0, 9), f32)
            self.mesh_normals = np.zeros((0, 3), f32)
        self.meshes = np.zeros(len(scene.Meshes), MESH_DTYPE)
        first = 0
        for i, m in enumerate(scene.Meshes):
            self.meshes[i]["first_triangle"] = first
            self.meshes[i]["triangle_count"] = len(m.Triangles)
            self.meshes[i]["material"] = m.MaterialData.record()
            self.meshes[i]["aabb"] = m.AABB
            first += len(m.Triangles)
        self.spheres = np.ascontiguousarray(scene.SphereData.Spheres, f32).reshape(-1, 4)
        self.sphere_materials = materials_array(scene.SphereData.Materials)
        self.point_lights = np.ascontiguousarray(scene.PointLights, f32).reshape(-1, 6)
        amb = np.asarray(scene.AmbientLight, f32)

        def ptr(a):
            return a.ctypes.data if a.size else None

        d = abi.rt_scene_desc()
        d.triangles = ptr(self.triangles)
        d.triangle_normals = ptr(self.triangle_normals)
        d.triangle_materials = ptr(self.triangle_materials)
        d.triangle_count = len(self.triangles)
        d.mesh_triangles = ptr(self.mesh_triangles)
        d.mesh_triangle_normals = ptr(self.mesh_normals)
        d.mesh_triangle_total = len(self.mesh_triangles)
        d.meshes = ptr(self.meshes)
        d.mesh_count = len(self.meshes)
        d.spheres = ptr(self.spheres)
        d.sphere_materials = ptr(self.sphere_materials)
        d.sphere_count = len(self.spheres)
        d.point_lights = ptr(self.point_lights)
        d.point_light_count = len(self.point_lights)
        d.ambient_radiance = abi.f3(amb)
        self.desc = d

    def ref(self):
        return C.byref(self.desc)
