"""The C-ABI library loads (no GPU needed), exports every entry point that
include/rt_mi355.h declares, and its struct layouts match the ctypes mirror.
No compute calls are made here."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_mi355.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rt_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_entry_points():
    names = _declared_functions()
    for n in ("rt_create", "rt_destroy", "rt_set_scene", "rt_render", "rt_render_device",
              "rt_last_error", "rt_intersect_rays", "rt_assemble_bands", "rt_abi_version",
              "rt_set_scene_ex", "rt_get_scene_info", "rt_set_scene_source", "rt_update_mesh_transforms",
              "rt_create_devices", "rt_get_device_info"):
        assert n in names


def test_library_exports_every_declared_symbol(rt):
    lib_path = rt.abi.LIB_PATH
    assert os.path.exists(lib_path), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [n for n in _declared_functions() if n not in exported]
    assert not missing, missing
    lib = rt.load_library()
    assert lib.rt_abi_version() == rt.abi.RT_ABI_VERSION
    for n in rt.abi.SIGNATURES:
        assert n in _declared_functions(), f"ctypes signature for undeclared {n}"


def test_ctypes_layouts(rt):
    a = rt.abi
    sizes = {
        a.rt_float3: 12, a.rt_triangle: 36, a.rt_sphere: 16, a.rt_aabb: 24, a.rt_material: 56,
        a.rt_point_light: 24, a.rt_camera: 48, a.rt_scene_info: 32, a.rt_mesh_source: 152, a.rt_image_plane: 20, a.rt_mesh: 88, a.rt_hit: 16,
        a.rt_ray: 24, a.rt_render_params: 40, a.rt_stats: 88, a.rt_device_info: 72,
    }
    for t, s in sizes.items():
        assert C.sizeof(t) == s, t.__name__


def test_c_layouts_match(tmp_path):
    """Compile a tiny C program against the header and compare sizeof/offsetof."""
    prog = tmp_path / "l.c"
    prog.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "rt_mi355.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(rt_material), sizeof(rt_mesh),
   sizeof(rt_scene_desc), sizeof(rt_render_params), sizeof(rt_stats), offsetof(rt_scene_desc, ambient_radiance),
   offsetof(rt_mesh, aabb), offsetof(rt_stats, kernel_ms), sizeof(rt_mesh_source),
   offsetof(rt_mesh_source, local_to_world), offsetof(rt_mesh_source, material), sizeof(rt_scene_info),
   offsetof(rt_stats, primary_scene_misses), sizeof(rt_device_info), offsetof(rt_stats, shadow_rays_moot));
 return 0; }''')
    exe = tmp_path / "l"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(prog)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    import _rt_pkg
    a = _rt_pkg.load().abi
    want = [C.sizeof(a.rt_material), C.sizeof(a.rt_mesh), C.sizeof(a.rt_scene_desc), C.sizeof(a.rt_render_params),
            C.sizeof(a.rt_stats), a.rt_scene_desc.ambient_radiance.offset, a.rt_mesh.aabb.offset,
            a.rt_stats.kernel_ms.offset, C.sizeof(a.rt_mesh_source), a.rt_mesh_source.local_to_world.offset,
            a.rt_mesh_source.material.offset, C.sizeof(a.rt_scene_info), a.rt_stats.primary_scene_misses.offset,
            C.sizeof(a.rt_device_info), a.rt_stats.shadow_rays_moot.offset]
    assert vals == want


def test_create_without_gpu_fails_loudly(rt):
    """On a machine without a gfx950 device the product path refuses to run
    (there is no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rt.RtError) as e:
        rt.Context()
    assert e.value.status in (rt.abi.RT_E_NO_DEVICE, rt.abi.RT_E_HIP)


def test_pixel_bytes_per_format(rt):
    """rt_pixel_bytes (host-only, no GPU needed): float RGBA 16, RGB32F 12,
    RGBA16F 8, RGBA8 4; and the Python flag constants equal the header's."""
    lib = rt.load_library()
    a = rt.abi
    assert [lib.rt_pixel_bytes(f) for f in (0, a.RT_FLAG_OUT_RGB32F, a.RT_FLAG_OUT_RGBA16F, a.RT_FLAG_OUT_RGBA8)] == \
        [16, 12, 8, 4]
    import re
    hdr = open(os.path.join(ROOT, "include", "rt_mi355.h")).read()
    for name, val in re.findall(r"#define (RT_(?:FLAG|GATHER|BUILD)_\w+)\s+(\d+)", hdr):
        assert getattr(a, name) == int(val), name
