"""Per-launch device time of one kernel instance from a rocprofv3 kernel trace.

    python tools/kt_span.py gpurun_out/kt_<tag> --kernel "render_kernel<false, false, false, true, 6, false>" --with sky_batch_kernel

With frames in flight (bench.py's four streams) the launches of the timed
instance overlap: each dispatch's own duration (rocprofv3 --stats "average")
includes the time it shares the CUs with its neighbours, so it exceeds the
time a launch costs the device.  This prints, for every kernel whose name
contains --kernel (or the largest one when omitted): the dispatch count, the
mean and median dispatch duration, and the union of the dispatch intervals
divided by the dispatch count — the device time per launch, the figure
bench.py's roofline uses (`roofline.avg_kernel_ms`: HIP events over the timed
frames / K); with --with (whole frames in flight: sky_batch_kernel after each
render_kernel) also the union over both kernels' launches per frame.  One JSON
line per kernel.
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import Counter, defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--with", dest="with_", default="",
                    help="a kernel launched once per frame beside --kernel (sky_batch_kernel): its last dispatches "
                         "join the union; the per-launch figure is per --kernel dispatch")
    ap.add_argument("--min-grid", type=int, default=0, help="ignore dispatches with a smaller grid (warm-up frames)")
    ap.add_argument("--last", type=int, default=0,
                    help="only the last N full-grid dispatches (bench.py --moving-frames 0: its timed frames are the "
                         "last launches of the in-flight instance)")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {a.trace_dir}")
    iv = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if a.kernel and a.kernel not in name and not (a.with_ and a.with_ in name):
                continue
            grid = int(float(row.get("Grid_Size") or row.get("Grid_Size_X") or 0))
            if grid < a.min_grid:
                continue
            iv[name].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), grid))

    def workload(lst):
        """the launches of the most frequent grid (not warm-up frames, not a
        stream's first frame before its order exists), the last --last"""
        freq = Counter(g for _, _, g in lst)
        grid = max(freq.items(), key=lambda gv: (gv[1], gv[0]))[0]
        out = sorted((s, e) for s, e, g in lst if g == grid)
        return grid, (out[-a.last:] if a.last else out)

    def union(lst):
        tot, cur_s, cur_e = 0, None, None
        for s, e in sorted(lst):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        return tot + (cur_e - cur_s if cur_e is not None else 0)

    mains = {k: v for k, v in iv.items() if not a.with_ or a.with_ not in k}
    comp = [v for k, v in iv.items() if a.with_ and a.with_ in k]
    for name, lst in sorted(mains.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        big, lst = workload(lst)
        durs = [(e - s) * 1e-6 for s, e in lst]
        line = {"kernel": name, "grid": big, "dispatches": len(lst),
                "mean_dispatch_ms": round(statistics.mean(durs), 5),
                "median_dispatch_ms": round(statistics.median(durs), 5),
                "union_ms_per_dispatch": round(union(lst) * 1e-6 / len(lst), 5)}
        if comp:
            # the companion's launches from the first of these on
            w = [(s, e) for c in comp for s, e, _ in c if s >= lst[0][0]]
            line.update({"with": a.with_, "with_dispatches": len(w),
                         "union_with_ms_per_dispatch": round(union(lst + w) * 1e-6 / len(lst), 5)})
        print(json.dumps(line))
        if not a.kernel:
            break


if __name__ == "__main__":
    main()
