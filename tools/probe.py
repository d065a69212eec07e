"""Perf probe: time render modes of one or more library variants on a config.

    python tools/probe.py --config C3 --variants default,bvh2 --frames 10
Variants are built by `make -C unity-raytracer_amd VARIANT=name EXTRA=...`.
Prints one JSON line per (variant, mode)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import _rt_pkg  # noqa: E402


def seg_per_wave(st):
    """RT_SEG_PROFILE words -> per-wave averages (64-sample waves)."""
    w = max(1, -(-st.primary_rays // 64))
    v = st.box_tests
    return {"waves": w, "nodes": round((v & 0xffffffff) / w, 2), "leaves": round((v >> 32) / w, 2),
            "prim_cyc": round(st.triangle_tests / w), "shadow_cyc": round(st.sphere_tests / w),
            "total_cyc": round(st.shading_fetches / w), "setup_cyc": round(st.primary_scene_misses / w)}


def seg_levels_per_wave(st, waves):
    """RT_SEG_PROFILE words of render_levels_kernel -> per-wave averages."""
    w = max(1, waves)
    se, mir = st.box_tests, st.primary_scene_misses
    setup, epi = (se & 0xffffffff) * 16, (se >> 32) * 16
    cam, sh, tot = st.triangle_tests, st.sphere_tests, st.shading_fetches
    return {"waves": w, "setup_cyc": round(setup / w), "cam_cyc": round(cam / w), "shadow_cyc": round(sh / w),
            "mirror_cyc": round(mir / w), "epilogue_cyc": round(epi / w), "total_cyc": round(tot / w),
            "shading_cyc": round((tot - setup - epi - cam - sh - mir) / w)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--variants", default="default")
    ap.add_argument("--modes", default="megakernel,packet,wavefront")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--res", default="")
    ap.add_argument("--bounces", type=int, default=-99)
    ap.add_argument("--no-lights", action="store_true")
    ap.add_argument("--band", default="", help="i/n: render only row band i of n (8-row blocks): a light load")
    ap.add_argument("--rgb32f", action="store_true", help="float RGB output (the bench's shard format at N > 1)")
    ap.add_argument("--async-frames", action="store_true",
                    help="timed frames with RT_FLAG_ASYNC, as bench.py times them")
    ap.add_argument("--streams", type=int, default=1,
                    help="--async-frames: rotate the frames over this many streams (frames in flight, as "
                         "bench.py's timed frames: a whole frame then runs the non-split instance; on one "
                         "stream it is a lone frame, which splits its slowest tiles)")
    a = ap.parse_args()
    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    if a.res:
        fr = fr.with_resolution(*map(int, a.res.split("x")))
    if a.spp:
        fr = fr.with_(spp=a.spp)
    if a.bounces != -99:
        fr = fr.with_(max_bounces=a.bounces)
    if a.no_lights:
        import numpy as np
        fr.scene.PointLights = np.zeros((0, 6), np.float32)
    base_img = None
    for v in a.variants.split(","):
        path = None if v == "default" else os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", v,
                                                         "librt_mi355.so")
        ctx = rt.Context(lib_path=path)
        ctx.set_scene(fr.scene)
        out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
        ref = None
        for mode in a.modes.split(","):
            flags = {"wavefront": rt.abi.RT_FLAG_WAVEFRONT, "packet": rt.abi.RT_FLAG_PACKET,
                     "rowmajor": rt.abi.RT_FLAG_ROW_ORDER}.get(mode, 0)
            if a.rgb32f:
                flags |= rt.abi.RT_FLAG_OUT_RGB32F
            bkw = {}
            if a.band:
                bi, bn = map(int, a.band.split("/"))
                bkw = dict(band_index=bi, band_count=bn, band_rows=8)
            p = rt.frame_params(fr, flags=flags, **bkw)
            cst = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=flags | 1, **bkw), out.data_ptr(),
                                    out.numel() * 4)
            img = out.cpu()
            same = None if ref is None else bool(torch.equal(img.view(torch.int32), ref.view(torch.int32)))
            ref = img if ref is None else ref
            base_img = img if base_img is None else base_img
            same_base = bool(torch.equal(img.view(torch.int32), base_img.view(torch.int32)))
            for _ in range(2):
                ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
            ks, ts = [], []
            if a.async_frames:
                pa = rt.frame_params(fr, flags=flags | rt.abi.RT_FLAG_ASYNC, **bkw)
                ss = [torch.cuda.Stream() for _ in range(max(1, a.streams))]
                oo = [out] + [torch.empty_like(out) for _ in ss[1:]]
                for k in range(a.frames):
                    ctx.set_stream(ss[k % len(ss)].cuda_stream)
                    ctx.render_device(fr.camera, fr.plane, pa, oo[k % len(ss)].data_ptr(), out.numel() * 4)
                st = ctx.finish()
                torch.cuda.synchronize()
                ctx.set_stream(None)
                for f_ in ("primary_rays", "shadow_rays", "reflection_rays"):
                    setattr(st, f_, getattr(st, f_) // a.frames)
                ks.append(st.kernel_ms / a.frames)
                ts.append(st.total_ms / a.frames)
            for _ in range(0 if a.async_frames else a.frames):
                st = ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
                ks.append(st.kernel_ms)
                ts.append(st.total_ms)
            rays = st.primary_rays + st.shadow_rays + st.reflection_rays
            km = statistics.median(ks)
            print(json.dumps({"variant": v, "mode": mode, "config": fr.name, "spp": fr.spp,
                              "bounces": fr.max_bounces, "lights": len(fr.scene.PointLights), "kernel_ms": round(km, 4),
                              "total_ms": round(statistics.median(ts), 4), "Mrays_s": round(rays / km / 1e3, 1),
                              "rays": rays, "box": cst.box_tests, "tri": cst.triangle_tests,
                              "sph": cst.sphere_tests, "same_as_first": same,
                              "same_as_base": same_base,
                              # RT_SEG_PROFILE builds: summed per-wave shader clocks (setup, camera packet,
                              # first shadow packet, whole tile) in the test-counter words of a timed frame
                              **({"seg_cycles": [st.box_tests, st.triangle_tests, st.sphere_tests,
                                                 st.shading_fetches],
                                  "seg_per_wave": seg_per_wave(st)} if "seg" in v and "seglv" not in v else {}),
                              # render_levels_kernel (>= 16 spp): one wave per 64 samples
                              **({"seg_levels_per_wave": seg_levels_per_wave(
                                  st, fr.plane.ResolutionX * fr.plane.ResolutionY * fr.spp // 64)}
                                 if "seglv" in v else {})}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
