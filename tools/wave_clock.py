"""Critical path of a render_kernel launch from per-wave clocks (a measuring
build: `make VARIANT=wclk EXTRA=-DRT_WAVE_CLOCK`; rt_debug_set
RT_DEBUG_WAVE_CLOCKS).  Each wave records its start and duration on the GPU's
constant 100 MHz clock; for the last launch of a run of synchronous frames (one
rank's row band 0/N, the bench's `--sim-bands N --streams 1` case) this prints
the launch's span, the slowest wave, when the last wave started (the end of
dispatch) and how much of the span the slowest waves cover.

    python tools/wave_clock.py --config C3 --bands 1,2,4,8 [--variant wclk] [--async-frames]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _rt_pkg  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def analyse(rec):
    """rec: (n, 4) uint32 records of one launch -> critical-path summary."""
    rec = rec[(rec[:, 0] | rec[:, 1] | rec[:, 2]) != 0]
    start = (rec[:, 1].astype(np.int64) << 32) | rec[:, 0].astype(np.int64)
    dur = rec[:, 2].astype(np.int64)
    t0 = start.min()
    s, e = start - t0, start - t0 + dur
    span = int(e.max())
    k = int(np.argmax(dur))
    part = (rec[:, 3] >> 24).astype(np.int64) - 1
    q = np.percentile(dur, [50, 90, 99, 99.9])
    order = np.sort(e)
    return {
        "waves": int(len(rec)),
        "span_us": round(span * TICK_US, 2),
        "last_start_us": round(int(s.max()) * TICK_US, 2),  # dispatch ends here
        "slowest_wave_us": round(int(dur[k]) * TICK_US, 2),
        "slowest_wave_start_us": round(int(s[k]) * TICK_US, 2),
        "slowest_wave_split": int(part[k]),  # -1 whole tile, else its quarter / sixteenth
        "slowest_wave_dispatch_rank": int(np.sum(s < s[k])),  # waves started before it
        "wave_us_p50_p90_p99_p999": [round(float(x) * TICK_US, 2) for x in q],
        "mean_wave_us": round(float(dur.mean()) * TICK_US, 2),
        "busy_wave_us": round(float(dur.sum()) * TICK_US, 1),
        "t_99pct_waves_done_us": round(int(order[int(0.99 * (len(order) - 1))]) * TICK_US, 2),
        "t_999pct_waves_done_us": round(int(order[int(0.999 * (len(order) - 1))]) * TICK_US, 2),
        "waves_running_at_90pct_span": int(np.sum((s <= 0.9 * span) & (e >= 0.9 * span))),
        "split_waves": int(np.sum(part >= 0)),
        "top_waves_us": [round(int(x) * TICK_US, 1) for x in np.sort(dur)[::-1][:16]],
        "top_waves_split": [int(part[i]) for i in np.argsort(dur)[::-1][:16]],
        # waves by duration (us bins): count and summed wave time — what the
        # short (sky) waves cost the launch against the long ones
        "dur_bins_us": [0, 2, 4, 8, 16, 32, 64, 128, 1e9],
        "dur_bin_waves": np.histogram(dur * TICK_US, [0, 2, 4, 8, 16, 32, 64, 128, 1e9])[0].tolist(),
        "dur_bin_busy_us": [round(float(dur[(dur * TICK_US >= lo) & (dur * TICK_US < hi)].sum()) * TICK_US, 1)
                            for lo, hi in zip([0, 2, 4, 8, 16, 32, 64, 128], [2, 4, 8, 16, 32, 64, 128, 1e9])],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--variant", default="wclk")
    ap.add_argument("--bands", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--async-frames", action="store_true",
                    help="RT_FLAG_ASYNC frames back to back on one stream (they split like synchronous ones)")
    a = ap.parse_args()
    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    path = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", a.variant, "librt_mi355.so")
    ctx = rt.Context(lib_path=path)
    lib = ctx.lib
    ctx.set_scene(fr.scene)
    assert lib.rt_debug_set(ctx.h, rt.abi.RT_DEBUG_WAVE_CLOCKS, 1) == 0, "not a RT_WAVE_CLOCK build"
    out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
    for n in map(int, a.bands.split(",")):
        bkw = dict(band_index=0, band_count=n, band_rows=8) if n > 1 else {}
        flags = rt.abi.RT_FLAG_OUT_RGB32F if n > 1 else 0
        if a.async_frames:
            flags |= rt.abi.RT_FLAG_ASYNC
        p = rt.frame_params(fr, flags=flags, **bkw)
        runs = []
        for f in range(a.frames):
            st = ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
            if a.async_frames:
                st = ctx.finish()
            if f < a.frames - 8:
                continue  # the longest-first order settles first
            buf = np.zeros(1 << 23, np.uint32)
            got = C.c_int64(0)
            assert lib.rt_debug_read(ctx.h, rt.abi.RT_DEBUG_WAVE_CLOCKS, buf.ctypes.data, buf.nbytes,
                                     C.byref(got)) == 0
            r = analyse(buf[: got.value // 4].reshape(-1, 4))
            r["kernel_ms_events"] = round(st.kernel_ms, 4)
            runs.append(r)
        med = sorted(runs, key=lambda r: r["span_us"])[len(runs) // 2]
        med.update({"config": fr.name, "band": f"0/{n}", "async": a.async_frames, "variant": a.variant,
                    "span_us_runs": [r["span_us"] for r in runs],
                    "slowest_wave_us_runs": [r["slowest_wave_us"] for r in runs],
                    "kernel_ms_median": round(statistics.median(r["kernel_ms_events"] for r in runs), 4)})
        print(json.dumps(med), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
