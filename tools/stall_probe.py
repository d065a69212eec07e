"""Stall probe for multi-device frames (round 4's two stalled GPU-suite runs).

Repeats what tests/test_gpu_multi.py's group tests do — 2/3/8-member logical
groups on one GPU, synchronous host frames (every member copies its own row
blocks into the caller's frame) and device frames (peer-copy gather +
reassembly), C1/C2/C3 scenes, every pixel format — for many rounds in one
process, optionally with one-sample split waves in the members' bands
(rt_debug_set RT_DEBUG_GROUP_SAMPLE_WAVES, the configuration both stalls ran
with).  Every frame must equal the one-device frame bit for bit.

A watchdog thread ends a stalled run: after --stall-s seconds without
progress it prints the library's host-wait report (which blocking call each
host thread sits in, rt_debug_read RT_DEBUG_HOST_WAITS), every open context's
stream states and every Python thread's stack, then exits with status 70.

usage (GPU box): python tools/stall_probe.py --rounds 40 [--sample-waves 1]
"""
import argparse
import faulthandler
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _rt_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--sample-waves", type=int, default=1)
    ap.add_argument("--stall-s", type=float, default=30.0)
    a = ap.parse_args()
    import torch

    rt = _rt_pkg.load()
    rtm = rt.raytracing
    last = [time.monotonic(), "start"]

    def watchdog():
        while True:
            time.sleep(1.0)
            if time.monotonic() - last[0] > a.stall_s:
                err = sys.__stderr__
                err.write(f"\n=== stall: no progress for {a.stall_s:.0f} s after '{last[1]}' ===\n")
                err.write(rtm.host_waits_report(None) + "\n")
                for c in list(rtm.LIVE_CONTEXTS):
                    if getattr(c, "h", None):
                        err.write(rtm.host_waits_report(c) + "\n")
                err.flush()
                faulthandler.dump_traceback(file=err, all_threads=True)
                err.flush()
                print(f"STALL after '{last[1]}'", flush=True)
                os._exit(70)

    threading.Thread(target=watchdog, daemon=True).start()

    def step(what):
        last[0] = time.monotonic()
        last[1] = what

    gpu = rt.Context()
    frames = {}
    for name, res, spp in (("C2", (333, 217), 4), ("C3", (480, 270), 4), ("C1", (97, 61), 1)):
        fr = rt.make(name).with_resolution(*res)
        frames[name] = fr.with_(spp=spp) if spp else fr
    c3s = [rt.make("C3").with_resolution(*r) for r in ((97, 61), (64, 8), (40, 3), (250, 131))]
    fmts = (0, rt.abi.RT_FLAG_OUT_RGBA8, rt.abi.RT_FLAG_OUT_RGB32F, rt.abi.RT_FLAG_OUT_RGBA16F)
    refs = {}
    for name, fr in frames.items():
        gpu.set_scene(fr.scene)
        refs[name] = gpu.render(fr.camera, fr.plane, rt.frame_params(fr))[0]
    for k, fr in enumerate(c3s):
        gpu.set_scene(fr.scene)
        for f in fmts:
            refs[("C3", k, f)] = gpu.render(fr.camera, fr.plane, rt.frame_params(fr, flags=f))[0]
    bad = 0
    t0 = time.monotonic()
    for rnd in range(a.rounds):
        for devs in ([0, 0], [0, 0, 0], [0] * 8):
            ctx = rt.Context(devices=devs, gather=1)
            if a.sample_waves:
                assert ctx.lib.rt_debug_set(ctx.h, rt.abi.RT_DEBUG_GROUP_SAMPLE_WAVES, 1) == 0
            try:
                for name, fr in frames.items():
                    step(f"round {rnd} group {len(devs)} {name} set_scene")
                    ctx.set_scene(fr.scene)
                    step(f"round {rnd} group {len(devs)} {name} render (host frame)")
                    img, _ = ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
                    bad += not np.array_equal(img.view(np.uint32), refs[name].view(np.uint32))
                    H, W = fr.plane.ResolutionY, fr.plane.ResolutionX
                    dev = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
                    step(f"round {rnd} group {len(devs)} {name} render_device")
                    ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr), dev.data_ptr(), dev.numel() * 4)
                    step(f"round {rnd} group {len(devs)} {name} device frame to host")
                    bad += not np.array_equal(dev.cpu().numpy().view(np.uint32), refs[name].view(np.uint32))
            finally:
                step(f"round {rnd} group {len(devs)} close")
                ctx.close()
        for n in (2, 3, 8):
            for k, fr in enumerate(c3s):
                ctx = rt.Context(devices=[0] * n, gather=1)
                if a.sample_waves:
                    assert ctx.lib.rt_debug_set(ctx.h, rt.abi.RT_DEBUG_GROUP_SAMPLE_WAVES, 1) == 0
                try:
                    step(f"round {rnd} direct {n} res {k} set_scene")
                    ctx.set_scene(fr.scene)
                    for f in fmts:
                        step(f"round {rnd} direct {n} res {k} flags {f} render")
                        img, _ = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=f))
                        bad += not np.array_equal(img.view(np.uint8), refs[("C3", k, f)].view(np.uint8))
                finally:
                    step(f"round {rnd} direct {n} res {k} close")
                    ctx.close()
        print(f"round {rnd}: ok, mismatching frames so far {bad}, {time.monotonic() - t0:.1f} s", flush=True)
    gpu.close()
    print(f"DONE rounds={a.rounds} sample_waves={a.sample_waves} mismatches={bad}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
