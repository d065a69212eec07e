"""Measurement only: C3 kernel time when the last N waves of the longest-first
order (sky tiles: key 0, dispatched last) are not launched — the upper bound
of what cheaper sky handling could save.  Also counts the frame's sky waves.
    python tools/exp/drop_tail.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _rt_pkg  # noqa: E402

rt = _rt_pkg.load()
fr = rt.make("C3")
ctx = rt.Context(lib_path=os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", "drop", "librt_mi355.so"))
ctx.set_scene(fr.scene)
out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
p = rt.frame_params(fr)
for drop in [0, 20000, 40000, 60000, 70000, 75000, 80000, 90000, 0]:
    os.environ["RT_EXP_DROP_TAIL"] = str(drop)
    for _ in range(3):
        ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
    ks = []
    for _ in range(15):
        st = ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
        ks.append(st.kernel_ms)
    print(json.dumps({"drop_waves": drop, "kernel_ms": round(statistics.median(ks), 4)}), flush=True)
