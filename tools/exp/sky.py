"""Cost of sky waves: C3 as is vs the camera turned around (every camera
sample misses Scene.AABB).  python tools/exp/sky.py"""
import json, os, statistics, sys
from dataclasses import replace
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa
import _rt_pkg  # noqa
rt = _rt_pkg.load()
fr = rt.make("C3")
c = fr.camera
back = replace(c, Forward=tuple(-v for v in c.Forward), Right=tuple(-v for v in c.Right))
var = sys.argv[1] if len(sys.argv) > 1 else ""
ctx = rt.Context(lib_path=os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", var, "librt_mi355.so")
                 if var else None)
ctx.set_scene(fr.scene)
out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
for name, cam in (("C3", c), ("sky", back)):
    p = rt.frame_params(fr)
    for _ in range(20):
        ctx.render_device(cam, fr.plane, p, out.data_ptr(), out.numel() * 4)
    ks = []
    for _ in range(20):
        st = ctx.render_device(cam, fr.plane, p, out.data_ptr(), out.numel() * 4)
        ks.append(st.kernel_ms)
    print(json.dumps({"variant": var or "default", "frame": name, "kernel_ms": statistics.median(ks), "primary": st.primary_rays,
                      "shadow": st.shadow_rays}), flush=True)
ctx.close()
