"""What the sky costs a frame in flight: C3 / C4 frames with the camera
turned away from the scene (every sample misses the scene box) against the
normal frames, four streams of RT_FLAG_ASYNC frames (measuring only)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import _rt_pkg  # noqa: E402

rt = _rt_pkg.load()
for name in sys.argv[1:] or ["C3", "C4"]:
    fr = rt.make(name)
    ctx = rt.Context()
    ctx.set_scene(fr.scene)
    c = fr.camera
    away = rt.CameraData(c.Position, tuple(-v for v in c.Forward), tuple(-v for v in c.Right), c.Up)
    H, W = fr.plane.ResolutionY, fr.plane.ResolutionX
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    p = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
    for label, cam in (("scene", c), ("sky", away), ("scene", c), ("sky", away)):
        n = 40 if name == "C3" else 12
        for rep in range(2):  # the first pass settles the longest-first state
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f in range(n):
                k = f % 4
                ctx.set_stream(streams[k].cuda_stream)
                ctx.render_device(cam, fr.plane, p, outs[k].data_ptr(), outs[k].numel() * 4)
            st = ctx.finish()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / n * 1e3
        print(name, label, round(ms, 4), "ms/frame", ctx.last_launch().split(" lpt")[0][-40:], flush=True)
    ctx.set_stream(None)
    ctx.close()
