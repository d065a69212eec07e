"""Host-side mirror of the reference's RayTracingSetup render interface.

The reference seam is the private ``RayTracingSetup.CastPixelRays(CameraData)``
(Assets/RayTracer/Demo-RayTracing/RayTracingSetup.cs:275-302), reading the
serialized fields ``ImagePlane`` (:21), ``BackgroundColor`` (:22),
``MaxReflectionBounces`` (:23) and ``Scene`` (:38) and writing
``PixelColors`` (:40).  ``RayTracingSetup`` below keeps those names and
meanings and drives the MI355X C-ABI (include/rt_mi355.h); there is no CPU
path: constructing it without the HIP library raises.
"""
from __future__ import annotations

import ctypes as C
import weakref
import math
from typing import Optional

import numpy as np

from . import abi
from .scene import Scene
from .scenes import CameraData, Frame, ImagePlane


def camera_struct(cam: CameraData) -> abi.rt_camera:
    return abi.rt_camera(abi.f3(cam.Position), abi.f3(cam.Forward), abi.f3(cam.Right), abi.f3(cam.Up))


def plane_struct(p: ImagePlane) -> abi.rt_image_plane:
    return abi.rt_image_plane(int(p.ResolutionX), int(p.ResolutionY), float(p.DistanceToCamera),
                              float(p.HalfHorizontalLength), float(p.HalfVerticalLength))


def channels(flags: int) -> int:
    """Channels per output pixel: 3 for RT_FLAG_OUT_RGB32F, else 4."""
    return 3 if flags & abi.RT_FLAG_OUT_RGB32F else 4


def pixel_dtype(flags: int):
    """numpy dtype of one output channel for rt_render_params.flags."""
    if flags & abi.RT_FLAG_OUT_RGBA8:
        return np.dtype(np.uint8)
    if flags & abi.RT_FLAG_OUT_RGBA16F:
        return np.dtype(np.float16)
    return np.dtype(np.float32)


def write_ppm(path: str, rgba8: np.ndarray):
    """Binary PPM (P6) of an RGBA8 frame (alpha dropped); y = 0 is the top
    row, as in PixelColors."""
    img = np.ascontiguousarray(np.asarray(rgba8, np.uint8)[..., :3])
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(img.tobytes())


def params_struct(background=(0, 0, 0, 1), max_bounces=0, spp=1, band_index=0, band_count=1,
                  band_rows=8, flags=0) -> abi.rt_render_params:
    p = abi.rt_render_params()
    for i in range(4):
        p.background_color[i] = float(background[i])
    p.max_reflection_bounces = int(max_bounces)
    p.samples_per_pixel = int(spp)
    p.band_index = int(band_index)
    p.band_count = int(band_count)
    p.band_rows = int(band_rows)
    p.flags = int(flags)
    return p


def frame_params(fr: Frame, **kw) -> abi.rt_render_params:
    return params_struct(fr.background, fr.max_bounces, kw.pop("spp", fr.spp), **kw)


# every open Context (the stall watchdogs report on them)
LIVE_CONTEXTS: "weakref.WeakSet[Context]" = weakref.WeakSet()


def host_waits_report(ctx=None, lib=None) -> str:
    """rt_debug_read(RT_DEBUG_HOST_WAITS): the library's host threads that sit
    in a blocking runtime call right now (which call, for how long) and, for a
    context, whether its streams still have work pending.  Callable from
    another thread while a call of that context is blocked (the watchdog of
    tests/conftest.py and tools/stall_probe.py)."""
    lib = lib or abi.load_library()
    buf = C.create_string_buffer(1 << 16)
    n = C.c_int64(0)
    h = ctx.h if ctx is not None else None
    st = lib.rt_debug_read(h, abi.RT_DEBUG_HOST_WAITS, C.cast(buf, C.c_void_p), len(buf), C.byref(n))
    return buf.value.decode(errors="replace") if st == abi.RT_OK else f"rt_debug_read: status {st}"


class Context:
    """Owns one rt_ctx.  Thin, error-checked wrapper of the C-ABI.

    num_gpus > 1 (or an explicit ``devices`` list, repeats = logical shards on
    one GPU) gives one context that renders every frame on all of them: row
    bands per device, gathered to devices[0] (RCCL or peer copies)."""

    def __init__(self, num_gpus: int = 1, lib_path: Optional[str] = None, devices=None, gather: int = 0):
        self.lib = abi.load_library(lib_path)
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            st = self.lib.rt_create_devices(C.byref(h), C.cast(arr, C.c_void_p), len(devices), int(gather))
        else:
            st = self.lib.rt_create(C.byref(h), int(num_gpus))
        if st != abi.RT_OK:
            raise abi.RtError(st, self.lib.rt_last_error(None).decode())
        self.h = h
        self._scene_desc = None
        LIVE_CONTEXTS.add(self)

    def _check(self, st: int):
        if st != abi.RT_OK:
            raise abi.RtError(st, self.lib.rt_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.rt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_info(self) -> dict:
        info = abi.rt_device_info()
        self._check(self.lib.rt_get_device_info(self.h, C.byref(info)))
        return {"num_devices": info.num_devices, "gather": info.gather,
                "devices": list(info.devices)[:min(16, info.num_devices)]}

    def last_launch(self) -> str:
        """The kernel instance of the context's last render launch and its
        split shape (rt_debug_read RT_DEBUG_LAST_LAUNCH)."""
        buf = C.create_string_buffer(512)
        n = C.c_int64(0)
        self._check(self.lib.rt_debug_read(self.h, abi.RT_DEBUG_LAST_LAUNCH, C.cast(buf, C.c_void_p), len(buf),
                                           C.byref(n)))
        return buf.value.decode()

    def set_stream(self, stream_handle: int):
        self._check(self.lib.rt_set_stream(self.h, C.c_void_p(stream_handle)))

    def set_scene(self, scene: Scene, build: Optional[int] = None):
        """Upload a scene and build its BVH: None = rt_set_scene's default (the
        on-device LBVH, 4-wide; the host SAH if that tree is too deep), or an
        explicit RT_BUILD_* through rt_set_scene_ex.  Renders are identical."""
        desc = scene.to_desc()
        if build is None:
            self._check(self.lib.rt_set_scene(self.h, desc.ref()))
        else:
            self._check(self.lib.rt_set_scene_ex(self.h, desc.ref(), int(build)))
        self._scene_desc = desc  # keep arrays alive for the duration of the call only; harmless

    def set_scene_source(self, base: Scene, sources, build: Optional[int] = None):
        """Device-side mesh extraction + GPU BVH build: `base` holds loose
        triangles, spheres and lights (no meshes); `sources` are MeshSource
        objects (local vertices, index buffer, localToWorld, material).
        build: None (rt_set_scene_source: a device LBVH rebuild per update) or
        abi.RT_BUILD_LBVH_GPU / abi.RT_BUILD_SAH_REFIT (rt_set_scene_source_ex)."""
        from .scene import MeshSourceArray
        if base.Meshes:
            raise ValueError("base scene must not carry extracted meshes")
        desc = base.to_desc()
        arr = MeshSourceArray(list(sources))
        if build is None:
            self._check(self.lib.rt_set_scene_source(self.h, desc.ref(), arr.ptr(), arr.count))
        else:
            self._check(self.lib.rt_set_scene_source_ex(self.h, desc.ref(), arr.ptr(), arr.count, int(build)))
        self._scene_desc = desc

    def update_mesh_transforms(self, local_to_world):
        """Per-frame transform update (mesh_count x 4 x 4 f32, row-major)."""
        m = np.ascontiguousarray(local_to_world, np.float32).reshape(-1, 16)
        self._check(self.lib.rt_update_mesh_transforms(self.h, m.ctypes.data if m.size else None, len(m)))

    def scene_info(self) -> dict:
        info = abi.rt_scene_info()
        self._check(self.lib.rt_get_scene_info(self.h, C.byref(info)))
        return info.as_dict()

    def render(self, camera: CameraData, plane: ImagePlane, params: abi.rt_render_params,
               out: Optional[np.ndarray] = None):
        rows = plane.ResolutionY
        if params.band_count > 1:
            rows = self.lib.rt_band_rows_local(plane.ResolutionY, params.band_index,
                                               params.band_count, params.band_rows)
        dtype = pixel_dtype(params.flags)
        ch = channels(params.flags)
        if out is None:
            out = np.empty((rows, plane.ResolutionX, ch), dtype)
        assert out.dtype == dtype and out.flags.c_contiguous and out.size >= rows * plane.ResolutionX * ch
        stats = abi.rt_stats()
        cam, pl = camera_struct(camera), plane_struct(plane)
        self._check(self.lib.rt_render(self.h, C.byref(cam), C.byref(pl), C.byref(params),
                                       out.ctypes.data_as(C.c_void_p), C.byref(stats)))
        return out, stats

    def render_device(self, camera, plane, params: abi.rt_render_params, dev_ptr: int, nbytes: int):
        """camera / plane: CameraData / ImagePlane, or prebuilt rt_camera /
        rt_image_plane structs (a frame loop builds them once)."""
        stats = abi.rt_stats()
        cam = camera if isinstance(camera, abi.rt_camera) else camera_struct(camera)
        pl = plane if isinstance(plane, abi.rt_image_plane) else plane_struct(plane)
        self._check(self.lib.rt_render_device(self.h, C.byref(cam), C.byref(pl), C.byref(params),
                                              C.c_void_p(dev_ptr), C.c_size_t(nbytes), C.byref(stats)))
        return stats

    def render_device_batch(self, cameras, plane, params: abi.rt_render_params, dev_ptr: int, stride: int):
        """rt_render_device_batch: len(cameras) frames of one layout as one
        launch, frame i at dev_ptr + i * stride (device memory)."""
        stats = abi.rt_stats()
        cams = (abi.rt_camera * len(cameras))(
            *[c if isinstance(c, abi.rt_camera) else camera_struct(c) for c in cameras])
        pl = plane if isinstance(plane, abi.rt_image_plane) else plane_struct(plane)
        self._check(self.lib.rt_render_device_batch(self.h, len(cameras), cams, C.byref(pl), C.byref(params),
                                                    C.c_void_p(dev_ptr), C.c_size_t(stride), C.byref(stats)))
        return stats

    def counter_words(self):
        """rt_debug_read(RT_DEBUG_COUNTERS): the 16 counter words of the last
        synchronous frame or rt_finish (word 9: fetched bytes, measuring
        builds)."""
        buf = (C.c_uint64 * 16)()
        n = C.c_int64(0)
        self._check(self.lib.rt_debug_read(self.h, abi.RT_DEBUG_COUNTERS, C.cast(buf, C.c_void_p), C.sizeof(buf),
                                           C.byref(n)))
        return list(buf)

    def finish(self) -> abi.rt_stats:
        """Wait for RT_FLAG_ASYNC frames; their summed stats."""
        stats = abi.rt_stats()
        self._check(self.lib.rt_finish(self.h, C.byref(stats)))
        return stats

    def assemble_bands(self, gathered_ptr: int, res_x: int, res_y: int, band_count: int,
                       band_rows: int, image_ptr: int, pixel_bytes: int = 16, sync: bool = True):
        """Reassemble gathered shards (device pointers); sync=False leaves the
        kernel stream-ordered on the context's stream."""
        self._check(self.lib.rt_assemble_bands_ex(self.h, C.c_void_p(gathered_ptr), res_x, res_y,
                                                  band_count, band_rows, pixel_bytes, C.c_void_p(image_ptr)))
        if sync:
            self._check(self.lib.rt_synchronize(self.h))

    def export_bvh(self):
        """The scene's 4-wide BVH as it lies in HBM (rt_export_bvh): node,
        triangle and sphere records as raw bytes (128 / 48 / 32 B each)."""
        info = abi.rt_bvh_export_info()
        self._check(self.lib.rt_export_bvh(self.h, None, None, None, C.byref(info)))
        nodes = np.zeros(info.nodes * 128, np.uint8)
        tris = np.zeros(info.triangle_records * 48, np.uint8)
        sphs = np.zeros(info.sphere_records * 32, np.uint8)
        self._check(self.lib.rt_export_bvh(self.h, nodes.ctypes.data_as(C.c_void_p), tris.ctypes.data_as(C.c_void_p),
                                           sphs.ctypes.data_as(C.c_void_p), C.byref(info)))
        return nodes, tris, sphs

    def intersect_rays(self, rays: np.ndarray) -> np.ndarray:
        """Scene.IntersectRay (Scene.cs:43-122) for (N, 6) float32 rays;
        returns a structured array (type, index, mesh_index, distance)."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        out = np.zeros(len(rays), HIT_DTYPE)
        self._check(self.lib.rt_intersect_rays(self.h, rays.ctypes.data_as(C.c_void_p), len(rays),
                                               out.ctypes.data_as(C.c_void_p)))
        return out


HIT_DTYPE = np.dtype([("type", np.int32), ("index", np.int32), ("mesh_index", np.int32),
                      ("distance", np.float32)])


class RayTracingSetup:
    """Mirror of RayTracingSetup's render part (RayTracingSetup.cs:19-40,275-302).

    Fields keep the reference's names: ImagePlane, BackgroundColor,
    MaxReflectionBounces, Scene, PixelColors.  SamplesPerPixel is the
    documented n*n extension (1 == reference)."""

    def __init__(self, scene: Scene, image_plane: ImagePlane, background_color=(0, 0, 0, 1),
                 max_reflection_bounces: int = 0, samples_per_pixel: int = 1,
                 context: Optional[Context] = None, build: int = abi.RT_BUILD_SAH_HOST):
        self.Scene = scene
        self.ImagePlane = image_plane
        self.BackgroundColor = tuple(background_color)
        self.MaxReflectionBounces = int(max_reflection_bounces)
        self.SamplesPerPixel = int(samples_per_pixel)
        self.PixelColors = np.zeros((0, 4), np.float32)
        self.ctx = context or Context()
        self.LastStats: Optional[abi.rt_stats] = None
        self.Build = int(build)
        self.UpdateScene()

    @classmethod
    def from_frame(cls, fr: Frame, context: Optional[Context] = None) -> "RayTracingSetup":
        return cls(fr.scene, fr.plane, fr.background, fr.max_bounces, fr.spp, context)

    def UpdateScene(self):
        """Upload Scene (replaces UpdateScene()'s result, :120-128; the
        library computes Scene.CalculateAABB and the BVH)."""
        self.ctx.set_scene(self.Scene, self.Build)

    def CastPixelRays(self, camera: CameraData, flags: int = 0) -> np.ndarray:
        """:275-302 — fills PixelColors (resX*resY RGBA, index x + y*resX)."""
        p = self.ImagePlane
        params = params_struct(self.BackgroundColor, self.MaxReflectionBounces, self.SamplesPerPixel,
                               flags=flags)
        img, stats = self.ctx.render(camera, p, params)
        self.PixelColors = img.reshape(-1, 4)
        self.LastStats = stats
        return self.PixelColors


def spp_side(spp: int) -> int:
    n = int(math.isqrt(spp))
    if n * n != spp or n < 1:
        raise ValueError(f"samples_per_pixel must be n*n, got {spp}")
    return n
