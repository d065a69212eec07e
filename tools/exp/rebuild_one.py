"""The shim's per-Update loop for a trace: rt_update_mesh_transforms + a frame, C3 knot spinning."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa
import _rt_pkg
from rebuild_bench import c3_sources
rt = _rt_pkg.load()
base, srcs, mats = c3_sources(rt)
out = torch.empty((base.plane.ResolutionY, base.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
p = rt.frame_params(base)
ctx = rt.Context()
ctx.set_scene_source(base.scene, srcs)
for k in range(12):
    t0 = time.perf_counter()
    ctx.update_mesh_transforms(mats(0.05 * k))
    t1 = time.perf_counter()
    st = ctx.render_device(base.camera, base.plane, p, out.data_ptr(), out.numel() * 4)
    t2 = time.perf_counter()
    print(k, round((t1 - t0) * 1e3, 4), round((t2 - t1) * 1e3, 4), round(st.kernel_ms, 4), flush=True)
