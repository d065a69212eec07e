"""Static-scene kernel time, host SAH tree vs device LBVH tree, each on a fresh
context (60 frames, median of the last 40), for C3 at depths 8 / 1 / 0 and C2."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa
import _rt_pkg
rt = _rt_pkg.load()
for name, bounces in (("C3", None), ("C3", 1), ("C3", 0), ("C2", None)):
    fr = rt.make(name)
    row = {"config": name, "bounces": bounces if bounces is not None else fr.max_bounces}
    out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
    for build in (0, 1):
        ctx = rt.Context()
        ctx.set_scene(fr.scene, build)
        p = rt.frame_params(fr)
        if bounces is not None:
            p.max_reflection_bounces = bounces
        ks = []
        for _ in range(60):
            st = ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)
            ks.append(st.kernel_ms)
        row[["sah", "lbvh"][build]] = round(statistics.median(ks[20:]), 4)
        ctx.close()
    row["gap"] = round(row["lbvh"] / row["sah"] - 1, 4)
    print(json.dumps(row), flush=True)
