"""Frames in flight on four streams: the sky tail each launch takes (RT_DEBUG_LAST_LAUNCH; measuring only)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, _rt_pkg
rt = _rt_pkg.load()
fr = rt.make("C3")
ctx = rt.Context()
ctx.set_scene(fr.scene)
ry, rx = fr.plane.ResolutionY, fr.plane.ResolutionX
outs = [torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda") for _ in range(4)]
streams = [torch.cuda.Stream() for _ in range(4)]
p = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
for f in range(80):
    k = f % 4
    ctx.set_stream(streams[k].cuda_stream)
    ctx.render_device(fr.camera, fr.plane, p, outs[k].data_ptr(), outs[k].numel() * 4)
    if f % 8 == 7:
        print(f, ctx.last_launch(), flush=True)
ctx.finish()
ctx.set_stream(streams[0].cuda_stream)
for f in range(6):
    ctx.render_device(fr.camera, fr.plane, p, outs[0].data_ptr(), outs[0].numel() * 4)
    print("one-stream", f, ctx.last_launch(), flush=True)
ctx.finish()
