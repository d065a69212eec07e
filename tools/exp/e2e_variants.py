"""rt_render (host output) end-to-end time of slab-weight variants (builds
with -DRT_EXP_SLAB_WEIGHTS=...), interleaved round by round.

    python tools/exp/e2e_variants.py --flags 8 --variants default,sw_1,sw_3_1 [--rounds 4]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import _rt_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--flags", type=int, default=8)
ap.add_argument("--variants", default="default")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--frames", type=int, default=10)
a = ap.parse_args()
rt = _rt_pkg.load()
fr = rt.make(a.config)
ry, rx = fr.plane.ResolutionY, fr.plane.ResolutionX
p = rt.frame_params(fr, flags=a.flags)
names = a.variants.split(",")
ctxs = {}
for v in names:
    path = None if v == "default" else os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", v, "librt_mi355.so")
    ctxs[v] = rt.Context(lib_path=path)
    ctxs[v].set_scene(fr.scene)
host = np.empty((ry, rx, rt.raytracing.channels(a.flags)), rt.raytracing.pixel_dtype(a.flags))
ref = None
ts = {v: [] for v in names}
same = {}
for _ in range(a.rounds):
    for v in names:
        for k in range(a.frames):
            t0 = time.perf_counter()
            ctxs[v].render(fr.camera, fr.plane, p, out=host)
            if k >= 2:
                ts[v].append(time.perf_counter() - t0)
        if ref is None:
            ref = host.copy()
        same[v] = bool(np.array_equal(ref.view(np.uint8), host.view(np.uint8)))
for v in names:
    print(json.dumps({"variant": v, "flags": a.flags, "e2e_ms": round(statistics.median(ts[v]) * 1e3, 4),
                      "min_ms": round(min(ts[v]) * 1e3, 4), "same_as_first": same[v]}), flush=True)
for c in ctxs.values():
    c.close()
