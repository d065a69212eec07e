"""ctypes wrapper of the CPU ORACLE (oracle/rt_oracle.c) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
this module; the product path (unity-raytracer_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

import unity_raytracer_amd as rt  # loaded by _rt_pkg.load_oracle()
from unity_raytracer_amd import abi
from unity_raytracer_amd.raytracing import HIT_DTYPE, camera_struct, plane_struct, params_struct

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class orc_counts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("primary_rays", "shadow_rays", "reflection_rays",
                                          "box_tests", "triangle_tests", "sphere_tests",
                                          "shading_fetches")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def default_threads() -> int:
    """Host threads for the oracle: OMP_NUM_THREADS (16 on the GPU box), capped at 16."""
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    return max(1, min(16, n))


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.orc_ray_aabb.argtypes = [P, P]
        L.orc_ray_triangle.argtypes = [P, P, C.POINTER(C.c_float)]
        L.orc_ray_sphere.argtypes = [P, P, C.POINTER(C.c_float)]
        L.orc_triangle_normal.argtypes = [P, P]
        L.orc_triangle_normal.restype = None
        L.orc_scene_aabb.argtypes = [P, P]
        L.orc_scene_aabb.restype = None
        L.orc_intersect.argtypes = [P, P, C.c_int32, P]
        L.orc_intersect.restype = None
        L.orc_render_pixels.argtypes = [P, P, P, P, P, C.c_int32, P, P, C.c_int32]
        L.orc_render_rows.argtypes = [P, P, P, P, C.c_int32, C.c_int32, P, P, C.c_int32]
        L.orc_render.argtypes = [P, P, P, P, P, P, C.c_int32]
        L.orc_spec_backfacing.argtypes = [C.c_float]
        L.orc_bvh_build.argtypes = [P]
        L.orc_bvh_build.restype = P
        L.orc_bvh_free.argtypes = [P]
        L.orc_bvh_free.restype = None
        L.orc_render_pixels_bvh.argtypes = [P, P, P, P, P, P, C.c_int32, P, P, C.c_int32]
        L.orc_bvh4_create.argtypes = [P, P, C.c_int32, P, C.c_int32, P, C.c_int32]
        L.orc_bvh4_create.restype = P
        L.orc_bvh4_free.argtypes = [P]
        L.orc_bvh4_free.restype = None
        L.orc_render_pixels_bvh4.argtypes = [P, P, P, P, P, P, C.c_int32, P, P, C.c_int32]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def ray_aabb(ray, box) -> bool:
    r = np.ascontiguousarray(ray, np.float32)
    b = np.ascontiguousarray(box, np.float32)
    return bool(lib().orc_ray_aabb(_p(r), _p(b)))


def ray_triangle(ray, tri):
    r = np.ascontiguousarray(ray, np.float32)
    t = np.ascontiguousarray(tri, np.float32)
    out = C.c_float(0)
    hit = bool(lib().orc_ray_triangle(_p(r), _p(t), C.byref(out)))
    return hit, np.float32(out.value)


def ray_sphere(ray, sph):
    r = np.ascontiguousarray(ray, np.float32)
    s = np.ascontiguousarray(sph, np.float32)
    out = C.c_float(0)
    hit = bool(lib().orc_ray_sphere(_p(r), _p(s), C.byref(out)))
    return hit, np.float32(out.value)


def triangle_normal(tri):
    t = np.ascontiguousarray(tri, np.float32)
    out = np.zeros(3, np.float32)
    lib().orc_triangle_normal(_p(t), _p(out))
    return out


def scene_aabb(scene: rt.Scene) -> np.ndarray:
    d = scene.to_desc()
    out = np.zeros(6, np.float32)
    lib().orc_scene_aabb(C.cast(d.ref(), C.c_void_p), _p(out))
    return out.reshape(2, 3)


def intersect(scene: rt.Scene, rays: np.ndarray) -> np.ndarray:
    d = scene.to_desc()
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    out = np.zeros(len(rays), HIT_DTYPE)
    lib().orc_intersect(C.cast(d.ref(), C.c_void_p), _p(rays), len(rays), _p(out))
    return out


def _frame_structs(fr, spp=None):
    cam = camera_struct(fr.camera)
    pl = plane_struct(fr.plane)
    prm = params_struct(fr.background, fr.max_bounces, fr.spp if spp is None else spp)
    return cam, pl, prm


def render(fr, threads: int = 0, spp=None):
    """Whole frame -> ((resY, resX, 4) f32, counts dict)."""
    d = fr.scene.to_desc()
    cam, pl, prm = _frame_structs(fr, spp)
    out = np.zeros((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), np.float32)
    cnt = orc_counts()
    st = lib().orc_render(C.cast(d.ref(), C.c_void_p), C.byref(cam), C.byref(pl), C.byref(prm),
                          _p(out), C.byref(cnt), threads or default_threads())
    if st != 0:
        raise RuntimeError(f"oracle render failed: {st}")
    return out, cnt.as_dict()


def render_pixels(fr, pixel_indices, threads: int = 0, spp=None):
    d = fr.scene.to_desc()
    cam, pl, prm = _frame_structs(fr, spp)
    idx = np.ascontiguousarray(pixel_indices, np.int32)
    out = np.zeros((len(idx), 4), np.float32)
    cnt = orc_counts()
    st = lib().orc_render_pixels(C.cast(d.ref(), C.c_void_p), C.byref(cam), C.byref(pl), C.byref(prm),
                                 _p(idx), len(idx), _p(out), C.byref(cnt), threads or default_threads())
    if st != 0:
        raise RuntimeError(f"oracle render failed: {st}")
    return out, cnt.as_dict()


class BvhScene:
    """A scene with a CPU BVH over it (CPU-baseline only: the same closest hits
    as the brute-force scan, found through a tree).  Keeps the descriptor and
    the tree alive; build time is spent here, outside any render timing."""

    def __init__(self, fr):
        self.fr = fr
        self.desc = fr.scene.to_desc()
        self.h = lib().orc_bvh_build(C.cast(self.desc.ref(), C.c_void_p))
        if not self.h:
            raise RuntimeError("oracle BVH build failed")

    def render_pixels(self, pixel_indices, threads: int = 0, spp=None):
        cam, pl, prm = _frame_structs(self.fr, spp)
        idx = np.ascontiguousarray(pixel_indices, np.int32)
        out = np.zeros((len(idx), 4), np.float32)
        cnt = orc_counts()
        st = lib().orc_render_pixels_bvh(self.h, C.cast(self.desc.ref(), C.c_void_p), C.byref(cam), C.byref(pl),
                                         C.byref(prm), _p(idx), len(idx), _p(out), C.byref(cnt),
                                         threads or default_threads())
        if st != 0:
            raise RuntimeError(f"oracle render failed: {st}")
        return out, cnt.as_dict()

    def close(self):
        if self.h:
            lib().orc_bvh_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Bvh4Scene:
    """A scene with the GPU's own 4-wide BVH (the byte records rt_export_bvh
    returns: 128-B nodes, 48-B triangle and 32-B sphere records), traversed on
    the CPU per ray like csrc/traverse.h (CPU-baseline only: the same tree as
    the GPU, so the algorithmic vs hardware split is like for like)."""

    def __init__(self, fr, nodes, tris, sphs):
        self.fr = fr
        self.desc = fr.scene.to_desc()
        self.keep = [np.ascontiguousarray(a, np.uint8) for a in (nodes, tris, sphs)]
        n, t, s = self.keep
        self.h = lib().orc_bvh4_create(C.cast(self.desc.ref(), C.c_void_p), _p(n), len(n) // 128, _p(t),
                                       len(t) // 48, _p(s), len(s) // 32)
        if not self.h:
            raise RuntimeError("oracle BVH4 create failed")

    def render_pixels(self, pixel_indices, threads: int = 0, spp=None):
        cam, pl, prm = _frame_structs(self.fr, spp)
        idx = np.ascontiguousarray(pixel_indices, np.int32)
        out = np.zeros((len(idx), 4), np.float32)
        cnt = orc_counts()
        st = lib().orc_render_pixels_bvh4(self.h, C.cast(self.desc.ref(), C.c_void_p), C.byref(cam), C.byref(pl),
                                          C.byref(prm), _p(idx), len(idx), _p(out), C.byref(cnt),
                                          threads or default_threads())
        if st != 0:
            raise RuntimeError(f"oracle render failed: {st}")
        return out, cnt.as_dict()

    def close(self):
        if self.h:
            lib().orc_bvh4_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def render_rows(fr, row_start, row_step, threads: int = 0, spp=None):
    d = fr.scene.to_desc()
    cam, pl, prm = _frame_structs(fr, spp)
    nrows = len(range(row_start, fr.plane.ResolutionY, row_step))
    out = np.zeros((nrows, fr.plane.ResolutionX, 4), np.float32)
    cnt = orc_counts()
    st = lib().orc_render_rows(C.cast(d.ref(), C.c_void_p), C.byref(cam), C.byref(pl), C.byref(prm),
                               row_start, row_step, _p(out), C.byref(cnt), threads or default_threads())
    if st != 0:
        raise RuntimeError(f"oracle render failed: {st}")
    return out, cnt.as_dict()


def spec_backfacing(d: float) -> bool:
    return bool(lib().orc_spec_backfacing(C.c_float(d)))
