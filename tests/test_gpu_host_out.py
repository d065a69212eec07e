"""rt_render into a host Color[] (rt_abi.cpp run_frame's slab pipeline): the
frame in row slabs that alternate over two streams, each slab copied to the
host once its launch ends while later slabs render.  The host frame must
equal the device frame (rt_render_device, then one copy) bit for bit — every
slab count, pixel format and spp — and stay equal over many frames of a
moving camera (each slab keeps its own longest-first order per stream)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F8, F16, F12 = 8, 16, 128


def _device_frame(ctx, fr, params, shape, dtype):
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    st = ctx.render_device(fr.camera, fr.plane, params, dev.data_ptr(), nbytes)
    return dev.cpu().numpy().view(dtype).reshape(shape), st


@pytest.mark.parametrize("flags", [0, F8, F16, F12])
def test_host_frame_equals_device_frame(gpu_ctx, rt, flags):
    fr = rt.make("C3")
    gpu_ctx.set_scene(fr.scene)
    p = rt.frame_params(fr, flags=flags)
    host, sh = gpu_ctx.render(fr.camera, fr.plane, p)
    ref, sd = _device_frame(gpu_ctx, fr, p, host.shape, host.dtype)
    assert np.array_equal(host.view(np.uint8), ref.view(np.uint8))
    assert (sh.primary_rays, sh.shadow_rays, sh.reflection_rays) == (sd.primary_rays, sd.shadow_rays,
                                                                     sd.reflection_rays)


@pytest.mark.parametrize("res,spp", [((1920, 1080), 1), ((1283, 719), 4), ((640, 997), 9), ((33, 7), 4),
                                     ((1, 1), 1), ((4096, 9), 4)])
def test_host_frame_shapes(gpu_ctx, rt, res, spp):
    """Slab counts 1..8, ragged last tile rows and columns, tiles of 64 / 16 /
    7 pixels (spp 1 / 4 / 9)."""
    fr = rt.make("C2").with_resolution(*res).with_(spp=spp)
    gpu_ctx.set_scene(fr.scene)
    p = rt.frame_params(fr)
    host, _ = gpu_ctx.render(fr.camera, fr.plane, p)
    ref, _ = _device_frame(gpu_ctx, fr, p, host.shape, host.dtype)
    assert np.array_equal(host.view(np.uint32), ref.view(np.uint32))


def _orbit(rt, cam0, n, yaw_deg=12.0):
    """CameraData of bench.orbit_cameras' moving views."""
    p0 = np.array(cam0.Position, np.float64)
    r = float(np.linalg.norm(p0))
    out = []
    for k in range(n):
        th = np.radians(yaw_deg) * np.sin(2 * np.pi * k / n)
        pos = np.array([-r * np.sin(th), p0[1], -r * np.cos(th)])
        fwd = -pos / np.linalg.norm(pos)
        right = np.cross([0.0, 1.0, 0.0], fwd)
        right /= np.linalg.norm(right)
        out.append(rt.CameraData(tuple(pos), tuple(fwd), tuple(right), tuple(np.cross(fwd, right))))
    return out


def test_host_frames_repeat_and_move(gpu_ctx, rt):
    """60 host frames of an orbiting camera into one array, checked against
    their device frames: every slab's copy waits for that frame's slab."""
    fr = rt.make("C3")
    gpu_ctx.set_scene(fr.scene)
    p = rt.frame_params(fr)
    cams = _orbit(rt, fr.camera, 6)
    host = np.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), np.float32)
    dev = torch.empty(host.nbytes, dtype=torch.uint8, device="cuda")
    for i in range(60):
        cam = cams[i % len(cams)]
        host[...] = np.nan
        gpu_ctx.render(cam, fr.plane, p, out=host)
        if i % 7 == 0 or i >= 56:
            gpu_ctx.render_device(cam, fr.plane, p, dev.data_ptr(), host.nbytes)
            ref = dev.cpu().numpy().view(np.uint32).reshape(host.shape)
            assert np.array_equal(host.view(np.uint32), ref), i


@pytest.mark.parametrize("fail_slab", [1, 3, 5])
def test_failed_slab_leaves_no_copy_behind(gpu_ctx, rt, fail_slab):
    """An error in a later slab (rt_debug_set RT_DEBUG_FAIL_SLAB injects one
    before that slab's launch) must not return before the copies already
    posted for the earlier slabs have finished: the caller may free or reuse
    its Color[] at once.  The earlier slabs' rows are the frame's, the rest
    of the buffer is untouched, nothing changes after the return, and the
    next frame succeeds with no error left behind."""
    import ctypes as C
    import time

    fr = rt.make("C3")  # float RGBA 1080p: six row slabs
    gpu_ctx.set_scene(fr.scene)
    p = rt.frame_params(fr)
    good, _ = gpu_ctx.render(fr.camera, fr.plane, p)
    lib = gpu_ctx.lib
    assert lib.rt_debug_set(gpu_ctx.h, rt.abi.RT_DEBUG_FAIL_SLAB, fail_slab) == 0
    try:
        buf = np.full(good.shape, -7.0, np.float32)
        stats = rt.abi.rt_stats()
        cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
        st = lib.rt_render(gpu_ctx.h, C.byref(cam), C.byref(pl), C.byref(p), buf.ctypes.data_as(C.c_void_p),
                           C.byref(stats))
        assert st == rt.abi.RT_E_INTERNAL
        assert b"slab" in lib.rt_last_error(gpu_ctx.h)
        snap = buf.copy()
        time.sleep(0.2)  # a copy still in flight would land now
        assert np.array_equal(snap.view(np.uint32), buf.view(np.uint32))
        done = np.all(buf == good, axis=(1, 2))      # rows the finished slabs copied
        untouched = np.all(buf == -7.0, axis=(1, 2))  # rows of the slabs never launched
        assert np.all(done | untouched)
        first_bad = int(np.argmin(done)) if not done.all() else len(done)
        assert 0 < first_bad < len(done) and untouched[first_bad:].all()
    finally:
        assert lib.rt_debug_set(gpu_ctx.h, rt.abi.RT_DEBUG_FAIL_SLAB, -1) == 0
    again, _ = gpu_ctx.render(fr.camera, fr.plane, p)
    assert np.array_equal(again.view(np.uint32), good.view(np.uint32))


def test_product_library_records_no_wave_clocks(gpu_ctx, rt):
    """RT_DEBUG_WAVE_CLOCKS belongs to measuring builds (-DRT_WAVE_CLOCK): the
    product library compiles no per-wave clock store and says so."""
    import ctypes as C

    lib = gpu_ctx.lib
    assert lib.rt_debug_set(gpu_ctx.h, rt.abi.RT_DEBUG_WAVE_CLOCKS, 1) == rt.abi.RT_E_STATE
    assert b"measuring" in lib.rt_last_error(gpu_ctx.h)
    n = C.c_int64(-1)
    buf = (C.c_uint32 * 4)()
    assert lib.rt_debug_read(gpu_ctx.h, rt.abi.RT_DEBUG_WAVE_CLOCKS, C.cast(buf, C.c_void_p), 16,
                             C.byref(n)) == rt.abi.RT_E_STATE
    assert n.value == 0
