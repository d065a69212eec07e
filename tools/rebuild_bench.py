"""Per-frame rebuild loop — the path the Unity shim runs every Update
(RayTracingSetup.cs:171-199: UpdateScene re-extracts every SceneMesh, then
CastPixelRays): rt_update_mesh_transforms (device extraction + GPU LBVH
rebuild) followed by a frame, against the same frames on a static host-SAH
scene and a static GPU-LBVH scene; then the same loop with the tree built once
on the host and refitted on the device per update (RT_BUILD_SAH_REFIT).

  python tools/rebuild_bench.py --config C3 --frames 40
C3: the torus-knot mesh as one SceneMesh spinning slowly about y; C5i: the
20,833 instanced boxes of scenes.instanced_hall, every box moving."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import _rt_pkg  # noqa: E402


def c3_sources(rt):
    fr = rt.make("C3")
    S = rt.scenes
    verts, idx = S.torus_knot()
    base = rt.Scene(TriangleData=fr.scene.TriangleData, Meshes=[], SphereData=fr.scene.SphereData,
                    PointLights=fr.scene.PointLights, AmbientLight=fr.scene.AmbientLight)
    c = np.array((0.0, -0.15, 0.15), np.float32)

    def matrices(t):
        q = S.yaw_quaternion(np.array([0.2 * t]))[0]
        m = rt.scene.quaternion_trs(np.zeros(3, np.float32), q, np.ones(3, np.float32)).astype(np.float32)
        m[:3, 3] = c - m[:3, :3] @ c  # spin about the knot's own center
        return m[None]

    src = [rt.MeshSource(verts, idx, matrices(0.0)[0], S.KNOT_MAT)]
    return fr.with_(scene=base), src, matrices


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=["C3", "C5i"])
    ap.add_argument("--frames", type=int, default=40)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    rt = _rt_pkg.load()
    if a.config == "C3":
        base, srcs, mats = c3_sources(rt)
    else:
        base, srcs, mats = rt.scenes.instanced_hall()
    ry, rx = base.plane.ResolutionY, base.plane.ResolutionX
    out = torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda")
    p = rt.frame_params(base)
    ctx = rt.Context()
    res = {"config": a.config, "frames": a.frames}

    # the matrices are made before the timed loop (C5i's are 20,833 Python-built TRS matrices)
    all_mats = [mats(0.05 * k) for k in range(a.frames + 3)]

    def frames(update):
        ks, ws = [], []
        for k in range(a.frames + 3):
            t0 = time.perf_counter()
            if update:
                ctx.update_mesh_transforms(all_mats[k])
            st = ctx.render_device(base.camera, base.plane, p, out.data_ptr(), out.numel() * 4)
            if k >= 3:
                ks.append(st.kernel_ms)
                ws.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(ks), 4), round(statistics.median(ws), 4)

    # static scenes: host SAH and GPU LBVH over the extracted meshes at t = 0
    fr0 = rt.scenes.extracted(base, srcs)
    for build, label in ((0, "static_sah"), (1, "static_lbvh")):
        ctx.set_scene(fr0.scene, build)
        res[label + "_kernel_ms"], res[label + "_wall_ms"] = frames(False)
    # per-frame device extraction + LBVH rebuild (the shim's Update)
    ctx.set_scene_source(base.scene, srcs)
    res["rebuild_kernel_ms"], res["rebuild_wall_ms"] = frames(True)
    info = ctx.scene_info()
    res["rebuild_update_ms"] = round(info["total_ms"], 4)
    res["rebuild_gpu_build_ms"] = round(info["build_ms"], 4)
    # RT_BUILD_SAH_REFIT (the C# shim's choice): host SAH tree once, refitted on the device every update
    ctx.set_scene_source(base.scene, srcs, build=rt.abi.RT_BUILD_SAH_REFIT)
    res["refit_kernel_ms"], res["refit_wall_ms"] = frames(True)
    info = ctx.scene_info()
    res["refit_update_ms"] = round(info["total_ms"], 4)
    res["refit_gpu_ms"] = round(info["build_ms"], 4)
    res["lbvh_gap"] = round(res["static_lbvh_kernel_ms"] / res["static_sah_kernel_ms"] - 1.0, 4)
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
