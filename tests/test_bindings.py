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
