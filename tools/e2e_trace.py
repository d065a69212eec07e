"""Timeline of rt_render's host-output path: where every
microsecond of a synchronous frame into a host Color[] / Color32[] goes.

    run (GPU box, under rocprofv3):
      rocprofv3 --runtime-trace --marker-trace --kernel-trace --memory-copy-trace --output-format csv -d DIR \\
          -o run -- python3 tools/e2e_trace.py run --flags 8 --frames 12
    analyse (anywhere):
      python3 tools/e2e_trace.py analyse DIR

`run` renders C3 frames with rt_render (synchronous, host output: the
library's row-slab pipeline, RayTracingSetup.cs:40,300 `PixelColors`); each
call is the library's roctx range "rt_render" in the marker trace, on the
profiler's clock.
`analyse` takes the median frame of the trace and attributes its wall time:
host time before the first launch, each slab's kernel span, each slab's copy
(the runtime's blit kernel `__amd_rocclr_copyBuffer` or an SDMA copy), the gaps
where neither a render kernel nor a copy runs, and the host tail after the
last copy (synchronisation, counter read).  Prints one JSON line.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(a):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch  # noqa: F401
    import _rt_pkg

    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    ctx = rt.Context()
    ctx.set_scene(fr.scene)
    p = rt.frame_params(fr, flags=a.flags)
    ch = 4
    host = np.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, ch), rt.raytracing.pixel_dtype(a.flags))
    out = []
    for k in range(a.frames):
        t0 = time.perf_counter()
        ctx.render(fr.camera, fr.plane, p, out=host)
        out.append(time.perf_counter() - t0)
    ctx.close()
    print(json.dumps({"flags": a.flags, "wall_ms": [round(t * 1e3, 4) for t in out]}))


def _rows(d, suffix):
    rows = []
    for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def _union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def analyse(a):
    frames = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in _rows(a.dir, "marker_api_trace.csv")
                    if any("rt_render" == str(v).strip() for v in r.values()))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in _rows(a.dir, "kernel_trace.csv")]
    cps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "")) for r in
           _rows(a.dir, "memory_copy_trace.csv")]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in _rows(a.dir, "hip_api_trace.csv")]
    res = []
    for t0, t1 in frames[2:]:  # the first frames allocate
        inside = lambda s, e: s >= t0 and e <= t1  # noqa: E731
        rk = [(s, e) for s, e, n in ks if inside(s, e) and "render" in n]
        blit = [(s, e) for s, e, n in ks if inside(s, e) and "copyBuffer" in n]
        other = [(s, e, n) for s, e, n in ks if inside(s, e) and "render" not in n and "copyBuffer" not in n]
        cp = [(s, e) for s, e, _ in cps if inside(s, e)]
        copies = blit + cp
        if not rk:
            continue
        first, last_r = min(s for s, _ in rk), max(e for _, e in rk)
        last_c = max((e for _, e in copies), default=last_r)
        busy = _union(rk + copies + [(s, e) for s, e, _ in other])
        sync = [(s, e, n) for s, e, n in api if s >= t0 and e <= t1 and "Synchronize" in n]
        res.append({
            "wall_us": (t1 - t0) / 1e3,
            "host_before_first_launch_us": (first - t0) / 1e3,
            "render_span_us": (last_r - first) / 1e3,
            "render_busy_us": _union(rk) / 1e3,
            "slab_kernels": len(rk),
            "copy_busy_us": _union(copies) / 1e3,
            "copies": len(copies),
            "copy_after_last_render_us": max(0, last_c - last_r) / 1e3,
            "other_kernels_us": _union([(s, e) for s, e, _ in other]) / 1e3,
            "other_kernels": sorted({n.split("(")[0][-40:] for _, _, n in other}),
            "device_idle_inside_us": ((last_c - first) - busy) / 1e3,
            "host_after_last_copy_us": (t1 - last_c) / 1e3,
            "sync_calls": len(sync),
        })
    res.sort(key=lambda r: r["wall_us"])
    med = res[len(res) // 2]
    num = {k: round(v, 1) for k, v in med.items() if isinstance(v, float)}
    print(json.dumps({"flags": a.flags, "frames": len(res), "median_frame": {**med, **num},
                      "wall_us_all": [round(r["wall_us"], 1) for r in res]}))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--config", default="C3")
    r.add_argument("--flags", type=int, default=8)
    r.add_argument("--frames", type=int, default=12)
    z = sub.add_parser("analyse")
    z.add_argument("dir")
    z.add_argument("--flags", type=int, default=8)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else analyse(a)


if __name__ == "__main__":
    main()
