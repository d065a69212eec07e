"""Timeline of bench.py's timed window from a rocprofv3 kernel trace.

    python tools/window_timeline.py gpurun_out/ktw_<tag> --steps 20

The timed frames are the last --steps dispatches of the in-flight render
instance (bench.py --moving-frames 0: the lone frames after the window run
another instance) and the sky / tally kernels between the first of them and
the window's last render end.  Prints one JSON line: the window's device span
(first timed start -> last timed kernel end) against K x the steady per-frame
period (the median start-to-start spacing of the timed renders), and how the
excess splits into fill (the first frames' starts before the queue is full),
drain (after the last render starts: its tail and its sky kernel) and the
time with fewer than `--low` kernels on the device.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--kernel", default="render_kernel<false, false, false, true, 6, false>")
    ap.add_argument("--lone", default="render_kernel<false, true, false, true, 6, false>")
    ap.add_argument("--low", type=int, default=2)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {a.trace_dir}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            grid = int(float(r.get("Grid_Size") or r.get("Grid_Size_X") or 0))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid,
                         (r.get("Stream_Id"), r.get("Queue_Id"))))
    rows.sort()
    sq = {(r[0], r[2]): r[4] for r in rows}
    rows = [r[:3] for r in rows]
    # the timed frames: the last --steps launches of the in-flight instance
    # before bench.py's lone frames (the longest run of back-to-back
    # --lone launches; rt_render's row slabs later run the in-flight
    # instance again)
    run, best, best_at = 0, 0, None
    for i, r in enumerate(rows):
        if a.lone in r[2]:
            run += 1
            if run > best:
                best, best_at = run, i - run + 1
        elif "render" in r[2]:
            run = 0
    if best_at is None:
        raise SystemExit(f"no {a.lone} launches")
    renders = [r for r in rows[:best_at] if a.kernel in r[2]]
    if len(renders) < a.steps:
        raise SystemExit(f"{len(renders)} dispatches of {a.kernel}")
    timed = renders[-a.steps:]
    t0 = timed[0][0]
    last_render_end = max(e for _, e, _ in timed)
    # the kernels of the window: everything that starts inside it up to the
    # last timed frame's tail kernels (sky batches / tallies), before the next render instance
    after = [r for r in rows if r[0] > timed[-1][0] and "render" in r[2]]
    stop = after[0][0] if after else float("inf")
    win = [r for r in rows if t0 <= r[0] < stop]
    t1 = max(e for _, e, _ in win)
    span = (t1 - t0) / 1e6
    starts = [s for s, _, _ in timed]
    gaps = [(b - c) / 1e6 for c, b in zip(starts, starts[1:])]
    period = statistics.median(gaps)
    # concurrency profile over the window
    ev = []
    for s, e, _ in win:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    active, prev, low_t, idle_t = 0, t0, 0.0, 0.0
    for t, d in ev:
        if t > prev:
            dt = (t - prev) / 1e6
            if active == 0:
                idle_t += dt
            elif active < a.low:
                low_t += dt
        active += d
        prev = t
    out = {
        "frames": len(timed),
        "span_ms": round(span, 4),
        "per_frame_ms": round(span / len(timed), 5),
        "median_start_spacing_ms": round(period, 5),
        "excess_over_K_periods_ms": round(span - period * len(timed), 4),
        "fill_ms": round((starts[min(len(starts) - 1, 7)] - t0) / 1e6, 4),
        "drain_after_last_start_ms": round((t1 - starts[-1]) / 1e6, 4),
        "last_render_to_end_ms": round((t1 - last_render_end) / 1e6, 4),
        "idle_ms": round(idle_t, 4),
        f"below_{a.low}_kernels_ms": round(low_t, 4),
        "stream_queue": sorted({"%s->%s" % sq[(s0, n)] for s0, _, n in timed}),
        "frame_ms": [round((e - s) / 1e6, 4) for s, e, _ in timed],
        "start_offsets_ms": [round((s - t0) / 1e6, 4) for s in starts],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
