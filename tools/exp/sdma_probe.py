"""Which HIP device-to-host copy calls run on the SDMA engines (not as blit
kernels that hold CU slots), their rate into a pageable host array, and what
a copy running beside a frame costs the frame.

    python tools/exp/sdma_probe.py --config C3
One JSON line per method: alone_ms (median), beside_ms (render + copy of the
previous frame started together, wall), kernel_ms beside."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _rt_pkg  # noqa: E402

D2H = 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    hip = C.CDLL("libamdhip64.so")
    for f in ("hipMemcpy", "hipMemcpyAsync", "hipMemcpyWithStream", "hipMemcpyDtoH", "hipStreamSynchronize",
              "hipDeviceSynchronize"):
        getattr(hip, f).restype = C.c_int
    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    ctx = rt.Context()
    ctx.set_scene(fr.scene)
    ry, rx = fr.plane.ResolutionY, fr.plane.ResolutionX
    nbytes = ry * rx * 16
    dev = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
    host = np.zeros(nbytes, np.uint8)
    s_render = torch.cuda.Stream()
    s_copy = torch.cuda.Stream()
    ctx.set_stream(s_render.cuda_stream)
    p = rt.frame_params(fr)
    pa = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
    for _ in range(3):
        ctx.render_device(fr.camera, fr.plane, p, dev[0].data_ptr(), nbytes)
    st = ctx.render_device(fr.camera, fr.plane, p, dev[1].data_ptr(), nbytes)
    kernel_alone = st.kernel_ms
    hp = host.ctypes.data
    cs = C.c_void_p(s_copy.cuda_stream)

    def copy(method, src):
        if method == "hipMemcpy":
            return hip.hipMemcpy(C.c_void_p(hp), C.c_void_p(src), C.c_size_t(nbytes), D2H)
        if method == "hipMemcpyDtoH":
            return hip.hipMemcpyDtoH(C.c_void_p(hp), C.c_void_p(src), C.c_size_t(nbytes))
        if method == "hipMemcpyWithStream":
            return hip.hipMemcpyWithStream(C.c_void_p(hp), C.c_void_p(src), C.c_size_t(nbytes), D2H, cs)
        if method == "hipMemcpyAsync":
            e = hip.hipMemcpyAsync(C.c_void_p(hp), C.c_void_p(src), C.c_size_t(nbytes), D2H, cs)
            return e or hip.hipStreamSynchronize(cs)
        raise ValueError(method)

    ref = dev[1].cpu().numpy()
    for method in ("hipMemcpy", "hipMemcpyDtoH", "hipMemcpyWithStream", "hipMemcpyAsync"):
        alone, beside, kb = [], [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            assert copy(method, dev[1].data_ptr()) == 0
            alone.append(time.perf_counter() - t0)
        ok = bool(np.array_equal(host, ref))
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.render_device(fr.camera, fr.plane, pa, dev[0].data_ptr(), nbytes)  # async frame
            assert copy(method, dev[1].data_ptr()) == 0  # the previous frame's pixels
            sf = ctx.finish()
            beside.append(time.perf_counter() - t0)
            kb.append(sf.kernel_ms)
        print(json.dumps({"method": method, "equal": ok, "kernel_alone_ms": round(kernel_alone, 4),
                          "copy_alone_ms": round(statistics.median(alone) * 1e3, 4),
                          "render_beside_copy_ms": round(statistics.median(beside) * 1e3, 4),
                          "kernel_beside_ms": round(statistics.median(kb), 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
