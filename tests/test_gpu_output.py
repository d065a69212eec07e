"""Output encoding on the device (RT_FLAG_OUT_RGBA8 / RT_FLAG_OUT_RGBA16F,
SURVEY §8(f) rank 3): the fused encode in the render kernel's final store
equals encoding the float frame (the reference's Color[] PixelColors) with
the restated Color -> Color32 / half conversions, for every render path, and
sharded frames reassemble in any format."""
import numpy as np
import pytest

import np_oracle as npo

pytestmark = pytest.mark.gpu

F8, F16, F12 = 8, 16, 128


@pytest.mark.parametrize("mode", [0, 2, 4])
def test_encoded_frames_equal_encoded_float_frame(gpu_ctx, rt, mode):
    fr = rt.make("C2").with_resolution(200, 113)
    gpu_ctx.set_scene(fr.scene)
    f, sf = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode))
    # push some channels outside [0, 1] to exercise the clamp: the lamp is > 1
    assert (f[..., :3] > 1.0).any() and (f[..., :3] == 0.0).any()
    b, sb = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode | F8))
    h, sh = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode | F16))
    assert b.dtype == np.uint8 and h.dtype == np.float16
    assert np.array_equal(b, npo.encode_rgba8(f))
    assert np.array_equal(h.view(np.uint16), npo.encode_rgba16f(f).view(np.uint16))
    assert (sf.primary_rays, sf.shadow_rays) == (sb.primary_rays, sb.shadow_rays) == (sh.primary_rays, sh.shadow_rays)


@pytest.mark.parametrize("flags,pb", [(F8, 4), (F16, 8), (F12, 12), (0, 16)])
def test_encoded_bands_reassemble(gpu_ctx, rt, flags, pb):
    import torch
    fr = rt.make("C2").with_resolution(150, 77)
    gpu_ctx.set_scene(fr.scene)
    full, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags))
    assert gpu_ctx.lib.rt_pixel_bytes(flags) == pb
    bands = 3
    parts = [gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=flags, band_index=k, band_count=bands))[0]
             for k in range(bands)]
    stacked = np.ascontiguousarray(np.stack(parts))
    gathered = torch.from_numpy(stacked.view(np.uint8).reshape(-1)).cuda()
    out = torch.empty(full.nbytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.assemble_bands(gathered.data_ptr(), fr.plane.ResolutionX, fr.plane.ResolutionY, bands, 8,
                           out.data_ptr(), pixel_bytes=pb)
    got = out.cpu().numpy().view(full.dtype).reshape(full.shape)
    assert np.array_equal(got.view(np.uint8), full.view(np.uint8))


@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rgb32f_is_the_float_frame_without_alpha(gpu_ctx, rt, mode):
    """RT_FLAG_OUT_RGB32F (the shard transport format): the Color values bit
    for bit, 12 B per pixel, for every render path and a >= 16 spp frame."""
    for fr in (rt.make("C2").with_resolution(120, 67), rt.make("C3").with_resolution(64, 36).with_(spp=16)):
        gpu_ctx.set_scene(fr.scene)
        f, sf = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode))
        c, sc = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode | F12))
        assert c.shape == f.shape[:2] + (3,) and c.dtype == np.float32
        assert np.array_equal(c.view(np.uint32), np.ascontiguousarray(f[..., :3]).view(np.uint32))
        assert (sf.primary_rays, sf.shadow_rays, sf.reflection_rays) == (sc.primary_rays, sc.shadow_rays,
                                                                         sc.reflection_rays)


def test_rgba8_ppm_writer(gpu_ctx, rt, tmp_path):
    fr = rt.make("demo")
    gpu_ctx.set_scene(fr.scene)
    b, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=F8))
    p = tmp_path / "demo.ppm"
    rt.write_ppm(str(p), b)
    data = p.read_bytes()
    assert data.startswith(b"P6\n50 50\n255\n") and len(data) == len(b"P6\n50 50\n255\n") + 50 * 50 * 3


def test_exclusive_formats(gpu_ctx, rt):
    fr = rt.make("C1").with_resolution(8, 8)
    gpu_ctx.set_scene(fr.scene)
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=F8 | F16))
    assert e.value.status == rt.abi.RT_E_INVALID
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=F12 | F16))
    assert e.value.status == rt.abi.RT_E_INVALID
