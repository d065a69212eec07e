"""End-to-end rt_render probe: synchronous frames into a host Color[] (pageable
or page-locked) against the kernel alone and the bare device-to-host copy.

    python tools/e2e_probe.py --config C3 --frames 12
Prints one JSON line per measurement (median over frames after the first)."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _rt_pkg  # noqa: E402


def med(ts):
    return round(statistics.median(ts[1:]) * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--variant", default="default")
    ap.add_argument("--mapped", action="store_true", help="also render straight into mapped page-locked memory")
    a = ap.parse_args()
    rt = _rt_pkg.load()
    fr = rt.make(a.config)
    path = None if a.variant == "default" else os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants",
                                                             a.variant, "librt_mi355.so")
    ctx = rt.Context(lib_path=path)
    ctx.set_scene(fr.scene)
    ry, rx = fr.plane.ResolutionY, fr.plane.ResolutionX
    p = rt.frame_params(fr, flags=a.flags)
    ch = rt.raytracing.channels(a.flags)
    dt = rt.raytracing.pixel_dtype(a.flags)
    nbytes = ry * rx * ch * np.dtype(dt).itemsize
    out = {"variant": a.variant, "config": fr.name, "flags": a.flags, "mbytes": round(nbytes / 1e6, 2)}
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ks = []
    for _ in range(a.frames):
        t0 = time.perf_counter()
        st = ctx.render_device(fr.camera, fr.plane, p, dev.data_ptr(), nbytes)
        ks.append(time.perf_counter() - t0)
    out["render_device_ms"] = med(ks)
    out["kernel_ms"] = round(st.kernel_ms, 4)
    for kind in ("pageable", "pinned"):
        if kind == "pinned":
            host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy().view(dt).reshape(ry, rx, ch)
        else:
            host = np.empty((ry, rx, ch), dt)
        host[...] = 0
        ts, tots = [], []
        for _ in range(a.frames):
            t0 = time.perf_counter()
            _, st = ctx.render(fr.camera, fr.plane, p, out=host)
            ts.append(time.perf_counter() - t0)
            tots.append(st.total_ms / 1e3)
        out[f"render_{kind}_ms"] = med(ts)
        ref = np.empty_like(host)
        torch.from_numpy(ref.reshape(-1).view(np.uint8)).copy_(dev.cpu())
        out[f"render_{kind}_equal"] = bool(np.array_equal(ref.view(np.uint32), host.view(np.uint32)))
        hs = torch.from_numpy(host.reshape(-1).view(np.uint8))
        cs = []
        for _ in range(a.frames):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hs.copy_(dev)
            cs.append(time.perf_counter() - t0)
        out[f"copy_{kind}_ms"] = med(cs)
    if a.mapped:
        # the kernel stores straight into page-locked host memory over PCIe
        # (rt_render_device with the pinned buffer's device address): no copy
        import ctypes as C
        lp = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
        hip = C.CDLL(lp)
        pinned = torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)
        dptr = C.c_void_p()
        rc = hip.hipHostGetDevicePointer(C.byref(dptr), C.c_void_p(pinned.data_ptr()), 0)
        out["mapped_rc"] = rc
        if rc == 0 and dptr.value:
            ms = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                st = ctx.render_device(fr.camera, fr.plane, p, dptr.value, nbytes)
                ms.append(time.perf_counter() - t0)
            out["render_mapped_ms"] = med(ms)
            out["render_mapped_kernel_ms"] = round(st.kernel_ms, 4)
            out["render_mapped_equal"] = bool(torch.equal(pinned, dev.cpu()))
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
