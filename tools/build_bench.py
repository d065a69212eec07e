"""Scene build cost per builder: rt_set_scene_ex wall time (upload + build),
GPU build kernel time (LBVH), and the frame time each BVH gives.

  python tools/build_bench.py --configs C2 C3 C5 --reps 5
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _rt_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C2", "C3", "C5"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--instanced", type=int, default=20833, help="instanced-hall boxes (0: skip)")
    ap.add_argument("--variant", default="", help="library variant under unity-raytracer_amd/lib/variants/")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    rt = _rt_pkg.load()
    lib = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", a.variant, "librt_mi355.so") if a.variant \
        else None
    ctx = rt.Context(lib_path=lib)
    for name in a.configs:
        fr = rt.make(name)
        for build, label in ((0, "sah_host_bvh4"), (1, "lbvh_gpu_bvh4"), (2, "lbvh_gpu_bvh2")):
            ctx.set_scene(fr.scene, build)  # warm (allocations, code objects)
            infos = []
            for _ in range(a.reps):
                ctx.set_scene(fr.scene, build)
                infos.append(ctx.scene_info())
            times = []
            out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
            for _ in range(a.frames):
                st = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr), out.data_ptr(), out.numel() * 4)
                times.append(st.kernel_ms)
            rec = {"config": name, "variant": a.variant or "default", "build": label, "primitives": infos[-1]["primitives"],
                   "nodes": infos[-1]["nodes"],
                   "set_scene_ms_min": min(i["total_ms"] for i in infos),
                   "gpu_build_ms_min": min(i["build_ms"] for i in infos),
                   "frame_ms_min": min(times)}
            print(json.dumps(rec), flush=True)
    if a.instanced:
        # device mesh extraction: C5-scale hall of 20,833 instanced cubes
        fr, srcs, mats = rt.scenes.instanced_hall(a.instanced)
        ctx.set_scene_source(fr.scene, srcs)
        first = ctx.scene_info()
        ms = [mats(0.1 * k) for k in range(a.reps + 1)]
        ctx.update_mesh_transforms(ms[0])  # warm
        infos, times = [], []
        for k in range(1, a.reps + 1):
            ctx.update_mesh_transforms(ms[k])
            infos.append(ctx.scene_info())
            out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
            st = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr), out.data_ptr(), out.numel() * 4)
            times.append(st.kernel_ms)
        print(json.dumps({"config": f"C5i ({a.instanced} instanced cubes, 1080p 4spp depth 8)",
                          "build": "device extraction + lbvh_gpu_bvh4",
                          "primitives": first["primitives"], "set_scene_source_ms": first["total_ms"],
                          "update_transforms_ms_min": min(i["total_ms"] for i in infos),
                          "update_gpu_ms_min": min(i["build_ms"] for i in infos),
                          "frame_ms_min": min(times)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
