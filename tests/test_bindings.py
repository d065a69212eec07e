"""The C# P/Invoke shim (bindings/csharp/, source only — no Mono here) names
exactly the entry points include/rt_mi355.h declares, and its blittable
structs list the same fields in the same order as the ctypes mirror whose
layout tests/test_abi.py checks against the C header."""
import os
import re

from test_abi import _declared_functions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "bindings", "csharp", "RtNative.cs")


def _dllimports():
    src = open(CS).read()
    names = set()
    for m in re.finditer(r"\[DllImport\(Lib(?:,\s*EntryPoint\s*=\s*\"(\w+)\")?\)\]\s*public static extern [\w.\[\]]+ (\w+)\(",
                         src):
        names.add(m.group(1) or m.group(2))
    return names


def test_shim_declares_every_entry_point():
    assert _dllimports() == set(_declared_functions())


def _cs_fields(struct):
    src = open(CS).read()
    body = re.search(r"public struct " + struct + r"\s*\{(.*?)\n    \}", src, re.S).group(1)
    body = re.sub(r"public static .*", "", body, flags=re.S)
    fields = []
    for decl in re.findall(r"public ([\w.]+) ([^;]+);", body):
        fields += [f.strip() for f in decl[1].split(",")]
    return fields


def test_shim_struct_field_counts(rt):
    a = rt.abi
    # (C# struct, ctypes struct, number of scalar-or-struct fields)
    for cs, ct in (("RtSceneDesc", a.rt_scene_desc), ("RtRenderParams", None), ("RtStats", a.rt_stats),
                   ("RtMeshSource", a.rt_mesh_source), ("RtSceneInfo", a.rt_scene_info),
                   ("RtImagePlane", a.rt_image_plane), ("RtMesh", a.rt_mesh), ("RtMaterial", a.rt_material)):
        got = _cs_fields(cs)
        if ct is None:  # background_color[4] is spelled out as four floats
            assert len(got) == 3 + len(a.rt_render_params._fields_)
            continue
        assert len(got) == len(ct._fields_), (cs, got)
    assert len(_cs_fields("RtMatrix")) == 16


SETUP = os.path.join(ROOT, "bindings", "csharp", "RayTracingSetupNative.cs")

# Every value the reference's per-Update scene fetch reads
# (RayTracingSetup.cs:120-169 and the SceneComponents getters), with the
# expression through which the shim reads it and the field of its StaticScene
# snapshot that carries it into the byte-for-byte change test.
REFERENCE_READS = [
    ("SceneTriangle.Triangle: position + Offset0/1/2 (SceneTriangle.cs:16-22)", "t.Triangle", "Tris"),
    ("SceneTriangle.Material (SceneTriangle.cs:12, FetchTriangles :166)", "Rt.Material(t.Material)", "TriMats"),
    ("SceneSphere.Sphere: position, localScale.x (SceneSphere.cs:9-22)", "x.Sphere", "Spheres"),
    ("SceneSphere.Material (SceneSphere.cs:7)", "Rt.Material(x.Material)", "SphMats"),
    ("ScenePointLight.Light: position + Intensity (ScenePointLight.cs:9-13)", "l.Light", "Lights"),
    ("SceneAmbientLight.AmbientLight (SceneAmbientLight.cs:7, :130-147)", "AmbientLight.Radiance", "Ambient"),
    ("number of ambient lights (:135-139)", "ambient.Length", "AmbientCount"),
    ("SceneMesh.MeshFilter.sharedMesh (SceneMesh.cs:15)", "m.MeshFilter.sharedMesh", "SharedMeshes"),
    ("Mesh.vertices (SceneMesh.cs:16)", "m.vertices", "Vertices"),
    ("Mesh.triangles (SceneMesh.cs:17)", "m.triangles", "Indices"),
    ("SceneMesh.Material (SceneMesh.cs:9)", "Rt.Material(m.Material)", "MeshMats"),
    ("the SceneMesh objects (FindObjectsOfType order)", "Meshes = meshes", "Meshes"),
]


def _method(src, name):
    i = src.index(name)
    j = src.index("{", i)
    depth, k = 0, j
    while True:
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
        k += 1


def test_shim_change_detection_covers_every_reference_read():
    """The shim re-sends the scene whenever anything the reference re-reads
    every Update changed: each read appears in UpdateScene's snapshot and each
    snapshot field in SameScene's comparison (localToWorldMatrix is uploaded
    every frame through rt_update_mesh_transforms)."""
    src = open(SETUP).read()
    update = _method(src, "void UpdateScene()")
    same = _method(src, "static bool SameScene(")
    for what, expr, field in REFERENCE_READS:
        assert expr in update, what
        assert f"a.{field}" in same and f"b.{field}" in same, what
    assert "localToWorldMatrix" in update and "rt_update_mesh_transforms" in update
    # byte-for-byte comparison (float bits), not float equality
    assert "MemoryMarshal.AsBytes" in src
