"""Host time of async frames on fresh streams (first use allocates the
stream's longest-first state): microseconds per rt_render_device call.

    python tools/first_frame.py [variant]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import _rt_pkg  # noqa: E402


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else ""
    rt = _rt_pkg.load()
    fr = rt.make("C3")
    ctx = rt.Context(lib_path=os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", lib, "librt_mi355.so")
                     if lib else None)
    s0 = torch.cuda.Stream()
    ctx.set_stream(s0.cuda_stream)
    ctx.set_scene(fr.scene)
    rx, ry = fr.plane.ResolutionX, fr.plane.ResolutionY
    out = torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda")
    cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
    prm = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
    streams = [s0] + [torch.cuda.Stream() for _ in range(3)]
    times = []
    # stream 0 keeps frames queued while streams 1-3 see their first frame
    for k in (0, 0, 0, 1, 0, 0, 2, 0, 0, 3, 1, 2, 3, 0):
        ctx.set_stream(streams[k].cuda_stream)
        t = time.perf_counter()
        ctx.render_device(cam, pl, prm, out.data_ptr(), out.numel() * 4)
        times.append((k, round((time.perf_counter() - t) * 1e6, 1)))
    ctx.finish()
    torch.cuda.synchronize()
    print(json.dumps({"host_us_per_frame": times}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
