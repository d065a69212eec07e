"""rt_render (host output) end-to-end time against slab weight vectors (RT_SLAB_WEIGHTS)."""
import json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa
import torch  # noqa
import _rt_pkg
rt = _rt_pkg.load()
fr = rt.make(sys.argv[1] if len(sys.argv) > 1 else "C3")
ctx = rt.Context()
ctx.set_scene(fr.scene)
ry, rx = fr.plane.ResolutionY, fr.plane.ResolutionX
W = {0: ["1", "1,1,1,1,1,1,1,1", "1,1,2,4,8", "1,2,4,8", "1,1,2,2,4,4", "1,2,3,4,6", "1,1,1,2,2,3,6", "1,2,2,3,3,4",
         "1,1,2,3,9"],
     8: ["1", "1,1,1", "1,1,1,1", "8,4,2,1", "4,2,1,1", "6,3,1", "2,2,1", "1,2,2,1", "3,3,2,1,1", "1,4,4,1"]}
for flags in (0, rt.abi.RT_FLAG_OUT_RGBA8):
    p = rt.frame_params(fr, flags=flags)
    host = np.empty((ry, rx, rt.raytracing.channels(flags)), rt.raytracing.pixel_dtype(flags))
    for w in W[flags]:
        os.environ["RT_SLAB_WEIGHTS"] = w
        ts, ks = [], []
        for k in range(16):
            t0 = time.perf_counter()
            _, st = ctx.render(fr.camera, fr.plane, p, out=host)
            ts.append(time.perf_counter() - t0)
            ks.append(st.kernel_ms)
        print(json.dumps({"flags": flags, "weights": w, "e2e_ms": round(statistics.median(ts[3:]) * 1e3, 4),
                          "min_ms": round(min(ts[3:]) * 1e3, 4),
                          "render_span_ms": round(statistics.median(ks[3:]), 4)}), flush=True)
