"""Host-side cost of the calls a frame loop makes per frame (render_device,
RCCL gather, wait, reassembly), one rank.  python tools/host_overhead.py"""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, torch.distributed as dist
import _rt_pkg
rt = _rt_pkg.load()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29577")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
fr = rt.make("C3")
ctx = rt.Context(); s = torch.cuda.current_stream(); ctx.set_stream(s.cuda_stream); ctx.set_scene(fr.scene)
out = torch.empty((1080, 1920, 4), device="cuda"); g = torch.empty((1, 1080, 1920, 4), device="cuda"); img = torch.empty_like(out)
p = rt.frame_params(fr, band_index=0, band_count=1, band_rows=8, flags=rt.abi.RT_FLAG_ASYNC)
def t(f, n=50):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): f()
    t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6
print("render_device host/total us", t(lambda: ctx.render_device(fr.camera, fr.plane, p, out.data_ptr(), out.numel() * 4)))
ctx.finish()
cs, ps = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
print("render_device prebuilt structs host/total us", t(lambda: ctx.render_device(cs, ps, p, out.data_ptr(), out.numel() * 4)))
ctx.finish()
pr = rt.frame_params(fr, band_index=0, band_count=1, band_rows=8, flags=rt.abi.RT_FLAG_ASYNC | rt.abi.RT_FLAG_ROW_ORDER)
print("render_device row-order host/total us", t(lambda: ctx.render_device(cs, ps, pr, out.data_ptr(), out.numel() * 4)))
ctx.finish()
print("gather async host/total us", t(lambda: dist.gather(out, list(g.unbind(0)), dst=0, async_op=True)))
w = dist.gather(out, list(g.unbind(0)), dst=0, async_op=True)
print("wait host us", t(lambda: w.wait()))
print("assemble host/total us", t(lambda: ctx.assemble_bands(g.data_ptr(), 1920, 1080, 1, 8, img.data_ptr(), sync=False)))
dist.destroy_process_group()
