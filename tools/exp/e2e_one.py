"""A few synchronous rt_render frames (host output) for a trace: python e2e_one.py <flags> <slabs> [frames]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa
import torch  # noqa
import _rt_pkg
os.environ["RT_SLABS"] = sys.argv[2]
rt = _rt_pkg.load()
fr = rt.make("C3")
ctx = rt.Context()
ctx.set_scene(fr.scene)
flags = int(sys.argv[1])
p = rt.frame_params(fr, flags=flags)
host = np.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, rt.raytracing.channels(flags)), rt.raytracing.pixel_dtype(flags))
for k in range(int(sys.argv[3]) if len(sys.argv) > 3 else 10):
    t0 = time.perf_counter()
    ctx.render(fr.camera, fr.plane, p, out=host)
    print(k, round((time.perf_counter() - t0) * 1e3, 4), flush=True)
