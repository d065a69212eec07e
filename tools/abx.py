"""Interleaved A/B of library variants in ONE process (drift-free comparison).

    python tools/abx.py --config C3 --variants base,default --rounds 12 --frames 10

Every variant's library is loaded side by side (lib/variants/<name>/ or the
default build), each with its own context and the scene resident; then for
`rounds` rounds every variant renders `frames` single frames (median
rt_stats.kernel_ms: one launch, HIP events) and `frames` asynchronous frames
on four streams (wall time per frame, the bench's mode), in a rotating order.
Prints one JSON line per variant with medians over rounds and the ratio to
the first variant; frames are checked bit-identical to the first variant's."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import torch  # noqa: E402
import _rt_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--variants", default="base,default")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--band", default="", help="i/n: row band i of n (one rank's share)")
    ap.add_argument("--flags", type=int, default=0)
    a = ap.parse_args()
    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    bkw = {}
    if a.band:
        bi, bn = map(int, a.band.split("/"))
        bkw = dict(band_index=bi, band_count=bn, band_rows=8)
    names = a.variants.split(",")
    H, W = fr.plane.ResolutionY, fr.plane.ResolutionX
    streams = [torch.cuda.Stream() for _ in range(4)]
    V = []
    for v in names:
        # "name@lbvh" / "name@sah": the same library with the scene built by the named builder
        # (no suffix: rt_set_scene's default)
        lib, _, build = v.partition("@")
        path = None if lib == "default" else os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", lib,
                                                           "librt_mi355.so")
        ctx = rt.Context(lib_path=path)
        ctx.set_scene(fr.scene, build={"lbvh": rt.abi.RT_BUILD_LBVH_GPU, "sah": rt.abi.RT_BUILD_SAH_HOST}.get(build))
        outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in streams]
        V.append({"name": v, "ctx": ctx, "outs": outs, "single": [], "stream": []})
    cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
    p = rt.frame_params(fr, flags=a.flags, **bkw)
    pa = rt.frame_params(fr, flags=a.flags | rt.abi.RT_FLAG_ASYNC, **bkw)
    nbytes = V[0]["outs"][0].numel() * 4
    # warm every variant (code objects, longest-first state on every stream) and check results
    ref = None
    for d in V:
        ctx = d["ctx"]
        for k, s in enumerate(streams):
            ctx.set_stream(s.cuda_stream)
            for _ in range(2):
                ctx.render_device(cam, pl, p, d["outs"][k].data_ptr(), nbytes)
        ctx.set_stream(streams[0].cuda_stream)
        torch.cuda.synchronize()
        img = d["outs"][0].cpu()
        if ref is None:
            ref = img
        d["same"] = bool(torch.equal(img.view(torch.int32), ref.view(torch.int32)))
    for r in range(a.rounds):
        order = V[r % len(V):] + V[:r % len(V)]
        for d in order:
            ctx = d["ctx"]
            ctx.set_stream(streams[0].cuda_stream)
            ks = []
            for _ in range(a.frames):
                st = ctx.render_device(cam, pl, p, d["outs"][0].data_ptr(), nbytes)
                ks.append(st.kernel_ms)
            d["single"].append(statistics.median(ks))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in range(a.frames):
                ctx.set_stream(streams[f % 4].cuda_stream)
                ctx.render_device(cam, pl, pa, d["outs"][f % 4].data_ptr(), nbytes)
            ctx.finish()
            torch.cuda.synchronize()
            d["stream"].append((time.perf_counter() - t0) / a.frames * 1e3)
            ctx.set_stream(streams[0].cuda_stream)
    b = V[0]
    bs, bt = statistics.median(b["single"]), statistics.median(b["stream"])
    for d in V:
        s, t = statistics.median(d["single"]), statistics.median(d["stream"])
        print(json.dumps({"variant": d["name"], "config": fr.name + (f" band {a.band}" if a.band else ""),
                          "single_ms": round(s, 4), "stream_ms": round(t, 4),
                          "single_vs_first": round(s / bs, 4), "stream_vs_first": round(t / bt, 4),
                          "single_spread": [round(min(d["single"]), 4), round(max(d["single"]), 4)],
                          "same_as_first": d["same"]}), flush=True)
    for d in V:
        d["ctx"].close()


if __name__ == "__main__":
    main()
