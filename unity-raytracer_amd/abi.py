"""ctypes mirror of include/rt_mi355.h (the C-ABI drop-in boundary).

Struct layouts are byte-for-byte those of the header; tests/test_abi.py checks
sizes and that the shared library exports every declared symbol.  The
library is the HIP build in ``unity-raytracer_amd/lib/librt_mi355.so``;
loading it never falls back to anything else — a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "librt_mi355.so")

RT_ABI_VERSION = 6
# earlier ABIs an A/B variant may have: version 5 lacks rt_render_device_batch only
OLDER_ABI_OK = (5,)
RT_MAX_BATCH = 8

RT_OK = 0
RT_E_INVALID = -1
RT_E_SCENE = -2
RT_E_HIP = -3
RT_E_NO_DEVICE = -4
RT_E_STATE = -5
RT_E_INTERNAL = -6

RT_FLAG_COUNT_TESTS = 1
RT_FLAG_WAVEFRONT = 2
RT_FLAG_PACKET = 4
RT_FLAG_OUT_RGBA8 = 8
RT_FLAG_OUT_RGBA16F = 16
RT_FLAG_OUT_RGB32F = 128
RT_FLAG_ASYNC = 32
RT_FLAG_ROW_ORDER = 64
RT_FLAG_NO_CUT = 256
RT_DEBUG_FAIL_SLAB = 1
RT_DEBUG_WAVE_CLOCKS = 2
RT_DEBUG_GROUP_SAMPLE_WAVES = 3
RT_DEBUG_HOST_WAITS = 4
RT_DEBUG_LAST_LAUNCH = 5
RT_DEBUG_SAMPLE_WAVE_STACK = 6
RT_DEBUG_COUNTERS = 7
RT_BUILD_SAH_HOST = 0
RT_BUILD_LBVH_GPU = 1
RT_BUILD_LBVH_GPU_BVH2 = 2
RT_BUILD_SAH_REFIT = 3  # rt_set_scene_source_ex: host SAH once, device refits per update
RT_GATHER_NONE = 0
RT_GATHER_PEER_COPY = 1
RT_GATHER_RCCL = 2

STATUS_NAMES = {
    RT_OK: "RT_OK",
    RT_E_INVALID: "RT_E_INVALID",
    RT_E_SCENE: "RT_E_SCENE",
    RT_E_HIP: "RT_E_HIP",
    RT_E_NO_DEVICE: "RT_E_NO_DEVICE",
    RT_E_STATE: "RT_E_STATE",
    RT_E_INTERNAL: "RT_E_INTERNAL",
}


class rt_float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class rt_triangle(C.Structure):
    _fields_ = [("vertex0", rt_float3), ("vertex1", rt_float3), ("vertex2", rt_float3)]


class rt_sphere(C.Structure):
    _fields_ = [("center", rt_float3), ("radius_squared", C.c_float)]


class rt_aabb(C.Structure):
    _fields_ = [("min", rt_float3), ("max", rt_float3)]


class rt_material(C.Structure):
    _fields_ = [
        ("diffuse_reflectance", rt_float3),
        ("ambient_reflectance", rt_float3),
        ("mirror_reflectance", rt_float3),
        ("specular_reflectance", rt_float3),
        ("phong_exponent", C.c_float),
        ("is_mirror", C.c_int32),
    ]


class rt_point_light(C.Structure):
    _fields_ = [("position", rt_float3), ("intensity", rt_float3)]


class rt_camera(C.Structure):
    _fields_ = [("position", rt_float3), ("forward", rt_float3), ("right", rt_float3), ("up", rt_float3)]


class rt_image_plane(C.Structure):
    _fields_ = [
        ("resolution_x", C.c_int32),
        ("resolution_y", C.c_int32),
        ("distance_to_camera", C.c_float),
        ("half_horizontal_length", C.c_float),
        ("half_vertical_length", C.c_float),
    ]


class rt_mesh(C.Structure):
    _fields_ = [
        ("first_triangle", C.c_int32),
        ("triangle_count", C.c_int32),
        ("material", rt_material),
        ("aabb", rt_aabb),
    ]


class rt_scene_desc(C.Structure):
    _fields_ = [
        ("triangles", C.c_void_p),
        ("triangle_normals", C.c_void_p),
        ("triangle_materials", C.c_void_p),
        ("triangle_count", C.c_int32),
        ("mesh_triangles", C.c_void_p),
        ("mesh_triangle_normals", C.c_void_p),
        ("mesh_triangle_total", C.c_int32),
        ("meshes", C.c_void_p),
        ("mesh_count", C.c_int32),
        ("spheres", C.c_void_p),
        ("sphere_materials", C.c_void_p),
        ("sphere_count", C.c_int32),
        ("point_lights", C.c_void_p),
        ("point_light_count", C.c_int32),
        ("ambient_radiance", rt_float3),
    ]


class rt_render_params(C.Structure):
    _fields_ = [
        ("background_color", C.c_float * 4),
        ("max_reflection_bounces", C.c_int32),
        ("samples_per_pixel", C.c_int32),
        ("band_index", C.c_int32),
        ("band_count", C.c_int32),
        ("band_rows", C.c_int32),
        ("flags", C.c_int32),
    ]


class rt_stats(C.Structure):
    _fields_ = [
        ("primary_rays", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("reflection_rays", C.c_uint64),
        ("box_tests", C.c_uint64),
        ("triangle_tests", C.c_uint64),
        ("sphere_tests", C.c_uint64),
        ("shading_fetches", C.c_uint64),
        ("kernel_ms", C.c_double),
        ("total_ms", C.c_double),
        ("primary_scene_misses", C.c_uint64),
        ("shadow_rays_moot", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class rt_device_info(C.Structure):
    _fields_ = [("num_devices", C.c_int32), ("gather", C.c_int32), ("devices", C.c_int32 * 16)]


class rt_mesh_source(C.Structure):
    _fields_ = [
        ("vertices", C.c_void_p),
        ("vertex_count", C.c_int32),
        ("indices", C.c_void_p),
        ("index_count", C.c_int32),
        ("local_to_world", C.c_float * 16),
        ("material", rt_material),
    ]


class rt_scene_info(C.Structure):
    _fields_ = [
        ("build", C.c_int32),
        ("bvh_width", C.c_int32),
        ("nodes", C.c_int32),
        ("primitives", C.c_int32),
        ("build_ms", C.c_double),
        ("total_ms", C.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class rt_hit(C.Structure):
    _fields_ = [("type", C.c_int32), ("index", C.c_int32), ("mesh_index", C.c_int32), ("distance", C.c_float)]


class rt_ray(C.Structure):
    _fields_ = [("origin", rt_float3), ("direction", rt_float3)]


class rt_bvh_export_info(C.Structure):
    _fields_ = [("nodes", C.c_int32), ("triangle_records", C.c_int32), ("sphere_records", C.c_int32),
                ("reserved", C.c_int32)]


# Every entry point declared in include/rt_mi355.h: name -> (restype, argtypes)
_P = C.c_void_p
SIGNATURES = {
    "rt_abi_version": (C.c_int32, []),
    "rt_create": (C.c_int, [C.POINTER(_P), C.c_int32]),
    "rt_create_devices": (C.c_int, [C.POINTER(_P), _P, C.c_int32, C.c_int32]),
    "rt_get_device_info": (C.c_int, [_P, C.POINTER(rt_device_info)]),
    "rt_destroy": (None, [_P]),
    "rt_last_error": (C.c_char_p, [_P]),
    "rt_set_stream": (C.c_int, [_P, _P]),
    "rt_set_scene": (C.c_int, [_P, C.POINTER(rt_scene_desc)]),
    "rt_set_scene_ex": (C.c_int, [_P, C.POINTER(rt_scene_desc), C.c_int32]),
    "rt_get_scene_info": (C.c_int, [_P, C.POINTER(rt_scene_info)]),
    "rt_export_bvh": (C.c_int, [_P, _P, _P, _P, C.POINTER(rt_bvh_export_info)]),
    "rt_set_scene_source": (C.c_int, [_P, C.POINTER(rt_scene_desc), _P, C.c_int32]),
    "rt_set_scene_source_ex": (C.c_int, [_P, C.POINTER(rt_scene_desc), _P, C.c_int32, C.c_int32]),
    "rt_update_mesh_transforms": (C.c_int, [_P, _P, C.c_int32]),
    "rt_render": (C.c_int, [_P, C.POINTER(rt_camera), C.POINTER(rt_image_plane),
                            C.POINTER(rt_render_params), _P, C.POINTER(rt_stats)]),
    "rt_render_device": (C.c_int, [_P, C.POINTER(rt_camera), C.POINTER(rt_image_plane),
                                   C.POINTER(rt_render_params), _P, C.c_size_t, C.POINTER(rt_stats)]),
    "rt_render_device_batch": (C.c_int, [_P, C.c_int32, _P, C.POINTER(rt_image_plane),
                                         C.POINTER(rt_render_params), _P, C.c_size_t, C.POINTER(rt_stats)]),
    "rt_band_rows_local": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rt_assemble_bands": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P]),
    "rt_pixel_bytes": (C.c_int32, [C.c_int32]),
    "rt_finish": (C.c_int, [_P, C.POINTER(rt_stats)]),
    "rt_synchronize": (C.c_int, [_P]),
    "rt_assemble_bands_ex": (C.c_int, [_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P]),
    "rt_intersect_rays": (C.c_int, [_P, _P, C.c_int32, _P]),
    "rt_debug_set": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "rt_debug_read": (C.c_int, [_P, C.c_int32, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
}

_lib = None


def load_library(path: str | None = None):
    """Load the HIP C-ABI library.  Raises if it is missing: there is no
    CPU fallback on the product path."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    # PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, but
    # torch links it as "libamdhip64.so").  Import torch first so this
    # library binds to the runtime torch uses, never a second copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise RuntimeError(
            f"rt_mi355 HIP library not found at {p}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = C.CDLL(p)
    # an explicitly named older build (a tools/abx.py or bench.py --lib A/B
    # variant) may lack later entry points: those stay unbound (AttributeError if used)
    older = path is not None and lib.rt_abi_version() in OLDER_ABI_OK
    for name, (res, args) in SIGNATURES.items():
        if (older or (path is not None and name.startswith("rt_debug"))) and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != RT_ABI_VERSION and not older:
        raise RuntimeError(f"rt_mi355 ABI mismatch: library {lib.rt_abi_version()} != {RT_ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


class RtError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


def f3(v) -> rt_float3:
    return rt_float3(float(v[0]), float(v[1]), float(v[2]))
