"""rt_render into a registered host buffer (rt_register_host_buffer): one
slab-major launch + copier_kernel streaming finished slabs over PCIe.  Every
frame must be bit-identical to the same frame rendered to device memory, with
the same ray counts — across consecutive frames (the longest-first order turns
slab-major after the first), every output format, non-2x2 sample layouts,
paths that fall back to render-then-copy, sub-ranges of the registered buffer
and frames after unregistering."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _device_frame(rt, ctx, fr, flags=0):
    ch = rt.raytracing.channels(flags)
    dt = rt.raytracing.pixel_dtype(flags)
    n = fr.plane.ResolutionY * fr.plane.ResolutionX * ch * np.dtype(dt).itemsize
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=flags), dev.data_ptr(), n)
    return dev.cpu().numpy().view(dt).reshape(fr.plane.ResolutionY, fr.plane.ResolutionX, ch), st


def _rays(st):
    return (st.primary_rays, st.shadow_rays, st.reflection_rays)


@pytest.mark.parametrize("name,res,spp", [("C2", None, 4), ("C3", None, 4), ("C2", (640, 360), 1),
                                          ("C3", (333, 211), 4), ("C2", (64, 48), 4), ("C1", None, 1)])
def test_registered_frames(rt, gpu_ctx, name, res, spp):
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=spp)
    gpu_ctx.set_scene(fr.scene)
    ref, rst = _device_frame(rt, gpu_ctx, fr)
    host = np.full((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), np.nan, np.float32)
    gpu_ctx.register_host_buffer(host)
    try:
        for k in range(4):  # frame 0 row-major, later frames slab-major longest-first
            host[...] = np.nan
            _, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr), out=host)
            assert np.array_equal(host.view(np.uint32), ref.view(np.uint32)), f"frame {k}"
            assert _rays(st) == _rays(rst)
    finally:
        gpu_ctx.unregister_host_buffer(host)


@pytest.mark.parametrize("flag", ["RT_FLAG_OUT_RGBA8", "RT_FLAG_OUT_RGBA16F", "RT_FLAG_OUT_RGB32F"])
def test_registered_formats(rt, gpu_ctx, flag):
    fr = rt.make("C2")
    flags = getattr(rt.abi, flag)
    gpu_ctx.set_scene(fr.scene)
    ref, _ = _device_frame(rt, gpu_ctx, fr, flags)
    host = np.zeros_like(ref)
    gpu_ctx.register_host_buffer(host)
    try:
        for _ in range(2):
            host[...] = 0
            gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags), out=host)
            assert np.array_equal(host, ref)
    finally:
        gpu_ctx.unregister_host_buffer(host)


@pytest.mark.parametrize("case", ["spp16_levels", "count_tests", "deep", "wavefront"])
def test_registered_fallback_paths(rt, gpu_ctx, orc, case):
    """Frames the streaming path does not take render first, then copy into the buffer."""
    fr = rt.make("C2").with_resolution(96, 54)
    flags = 0
    if case == "spp16_levels":
        fr = fr.with_(spp=16)
    elif case == "count_tests":
        flags = rt.abi.RT_FLAG_COUNT_TESTS
    elif case == "deep":
        fr = rt.scenes.mirror_corridor(40)
    else:
        flags = rt.abi.RT_FLAG_WAVEFRONT
    gpu_ctx.set_scene(fr.scene)
    ref, _ = orc.render(fr)
    host = np.full((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), np.nan, np.float32)
    gpu_ctx.register_host_buffer(host)
    try:
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags), out=host)
    finally:
        gpu_ctx.unregister_host_buffer(host)
    assert np.max(np.abs(host - ref)) <= 1e-4


def test_registered_subrange_resolution_changes_and_unregister(rt, gpu_ctx):
    """One large registered buffer serves frames of several sizes (a prefix of
    it); after unregistering, the same array renders through the copy path."""
    fr = rt.make("C3")
    gpu_ctx.set_scene(fr.scene)
    big = np.zeros(1920 * 1080 * 4, np.float32)
    gpu_ctx.register_host_buffer(big)
    try:
        for rx, ry in ((1920, 1080), (800, 600), (1920, 1080), (37, 1000)):
            f = fr.with_resolution(rx, ry)
            ref, _ = _device_frame(rt, gpu_ctx, f)
            view = big[:ry * rx * 4].reshape(ry, rx, 4)
            gpu_ctx.render(f.camera, f.plane, rt.frame_params(f), out=view)
            assert np.array_equal(view.view(np.uint32), ref.view(np.uint32)), (rx, ry)
        with pytest.raises(rt.RtError):
            gpu_ctx.register_host_buffer(big[:1024])  # overlaps
    finally:
        gpu_ctx.unregister_host_buffer(big)
    with pytest.raises(rt.RtError):
        gpu_ctx.unregister_host_buffer(big)  # no longer registered
    ref, _ = _device_frame(rt, gpu_ctx, fr)
    view = big.reshape(1080, 1920, 4)
    view[...] = 0
    gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr), out=view)
    assert np.array_equal(view.view(np.uint32), ref.view(np.uint32))
