"""rt_render (host output) end-to-end time against the row-slab count
(RT_SLABS, read by the library per frame): float RGBA and RGBA8."""
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
for flags in (0, rt.abi.RT_FLAG_OUT_RGBA8):
    p = rt.frame_params(fr, flags=flags)
    host = np.empty((ry, rx, rt.raytracing.channels(flags)), rt.raytracing.pixel_dtype(flags))
    for ns in (1, 2, 3, 4, 6, 8, 12, 16):
        os.environ["RT_SLABS"] = str(ns)
        ts = []
        for k in range(14):
            t0 = time.perf_counter()
            ctx.render(fr.camera, fr.plane, p, out=host)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"flags": flags, "slabs": ns, "e2e_ms": round(statistics.median(ts[2:]) * 1e3, 4),
                          "min_ms": round(min(ts[2:]) * 1e3, 4)}), flush=True)
    src = torch.empty(host.nbytes, dtype=torch.uint8, device="cuda")
    hs = torch.from_numpy(host.view(np.uint8).reshape(-1))
    cs = []
    for _ in range(8):
        torch.cuda.synchronize(); t0 = time.perf_counter(); hs.copy_(src); cs.append(time.perf_counter() - t0)
    print(json.dumps({"flags": flags, "bare_copy_ms": round(statistics.median(cs[2:]) * 1e3, 4)}), flush=True)
