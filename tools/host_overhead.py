"""Host cost of each call in bench.py's distributed frame loop (one rank,
RCCL process group of size 1): microseconds per call, GPU work async.

    python tools/host_overhead.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _rt_pkg  # noqa: E402


def per_call_us(fn, n=200):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return round(dt, 1)


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    rt = _rt_pkg.load()
    fr = rt.make("C3")
    ctx = rt.Context()
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    ctx.set_scene(fr.scene)
    rx, ry = fr.plane.ResolutionX, fr.plane.ResolutionY
    rows = ctx.lib.rt_band_rows_local(ry, 0, 8, 8)
    out = torch.empty((rows, rx, 3), dtype=torch.float32, device="cuda")
    gath = torch.empty((1, rows, rx, 3), dtype=torch.float32, device="cuda")
    img = torch.empty((ry, rx, 3), dtype=torch.float32, device="cuda")
    lst = list(gath.unbind(0))
    cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
    prm = rt.frame_params(fr, band_index=0, band_count=8, band_rows=8,
                          flags=rt.abi.RT_FLAG_OUT_RGB32F | rt.abi.RT_FLAG_ASYNC)
    r = {}
    with torch.cuda.stream(s):
        r["render_device"] = per_call_us(lambda: ctx.render_device(cam, pl, prm, out.data_ptr(), out.numel() * 4), 100)
        ctx.finish()
        r["gather_async"] = per_call_us(lambda: dist.gather(out, lst, dst=0, async_op=True).wait())
        r["gather_list_build"] = per_call_us(lambda: list(gath.unbind(0)))
        # one band of the full height (band_count 1): the source holds ry rows
        full = torch.empty((1, ry, rx, 3), dtype=torch.float32, device="cuda")
        assert full.numel() == img.numel()
        r["assemble"] = per_call_us(lambda: ctx.assemble_bands(full.data_ptr(), rx, ry, 1, 8, img.data_ptr(),
                                                               pixel_bytes=12, sync=False))
        r["set_stream"] = per_call_us(lambda: ctx.set_stream(s.cuda_stream))

    def stream_ctx():
        with torch.cuda.stream(s):
            pass
    r["torch_stream_ctx"] = per_call_us(stream_ctx)
    print(json.dumps({"host_us_per_call": r}), flush=True)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
