"""Fetched bytes per frame of the bench's timed path, from the measuring build
lib/variants/fetch (make VARIANT=fetch EXTRA=-DRT_FETCH_COUNT; traverse.h
RT_FETCH_*): the bytes a frame's traversal and shading request from the
cache hierarchy — each node, primitive, gate, cut and shading record a packet
fetches by scalar loads counted once per wave, each one a lane fetches by
itself (mirror chains) once per lane — where SURVEY §8(d)'s logical bytes
price every per-lane test (VERDICT r05 "Next" item 7).

    python tools/fetch_bytes.py [--configs C2,C3,C4,C5] [--out profiles/canonical_counts.json]

Runs on the GPU box.  Frames as bench.py times them: four streams of
RT_FLAG_ASYNC frames in flight after one setup frame per stream (whole
frames in flight never split their tiles, so the count is a function of the
tree and the camera); a lone synchronous frame (the split instance) is
reported beside it.  Adds `fetched_bytes_per_frame` (and `_lone`) to each
config's entry of the canonical-counts file; bench.py reports the committed
figure as roofline.fetched_bytes_per_launch and re-measures it when the
variant library is present."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _rt_pkg  # noqa: E402

VARIANT = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", "fetch", "librt_mi355.so")


def timed_path_fetch(rt, fr, lib_path=VARIANT, frames=8, streams=4):
    """(fetched bytes per in-flight frame, per lone frame, last launch) of fr."""
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    ctx = rt.Context(lib_path=lib_path)
    ss = [torch.cuda.Stream() for _ in range(streams)]
    try:
        ctx.set_stream(ss[0].cuda_stream)
        ctx.set_scene(fr.scene)
        outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in ss]
        nbytes = outs[0].numel() * 4
        p = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
        cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
        for k in range(2 * streams):  # setup: every stream's order and sky tail measured and known
            ctx.set_stream(ss[k % streams].cuda_stream)
            ctx.render_device(cam, pl, p, outs[k % streams].data_ptr(), nbytes)
        ctx.finish()
        torch.cuda.synchronize()
        for f in range(frames):
            ctx.set_stream(ss[f % streams].cuda_stream)
            ctx.render_device(cam, pl, p, outs[f % streams].data_ptr(), nbytes)
        launch = ctx.last_launch()
        ctx.finish()
        words = ctx.counter_words()
        torch.cuda.synchronize()
        ctx.set_stream(None)
        for _ in range(2):  # the second lone frame splits by the first's order
            ctx.render_device(cam, pl, rt.frame_params(fr), outs[0].data_ptr(), nbytes)
        lone = ctx.counter_words()[9]
    finally:
        ctx.set_stream(None)
        ctx.close()
    return words[9] / frames, lone, launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C3,C4,C5")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "canonical_counts.json"))
    a = ap.parse_args()
    if not os.path.exists(VARIANT):
        raise SystemExit(f"build the measuring variant first: make -C unity-raytracer_amd VARIANT=fetch "
                         f"EXTRA=-DRT_FETCH_COUNT ({VARIANT} missing)")
    rt = _rt_pkg.load()
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for name in a.configs.split(","):
        fr = rt.make(name)
        per_frame, lone, launch = timed_path_fetch(rt, fr)
        e = res.setdefault(name, {"config": name})
        e["fetched_bytes_per_frame"] = per_frame
        e["fetched_bytes_lone_frame"] = lone
        e["fetched_launch"] = launch.split(" lpt:")[0]
        print(json.dumps({"config": name, "fetched_bytes_per_frame": per_frame, "lone": lone,
                          "launch": e["fetched_launch"]}), flush=True)
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
