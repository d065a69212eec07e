"""Canonical per-frame test counts of the BASELINE configs at
full size, from the CPU oracle's walk of the GPU's exported 4-wide tree
(oracle/rt_oracle.c bvh4_query), checked against the GPU counting launch
(RT_FLAG_COUNT_TESTS) of the same frame — they must be equal.

    python tools/canonical_counts.py [--configs C2,C3] [--out profiles/canonical_counts.json]

Runs on the GPU box (the tree is built by the library).  bench.py prices
`roofline.logical_bytes_per_launch` from its own counting launch and reports
whether it equals the figure committed here (`canonical_counts: match`)."""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import _rt_pkg  # noqa: E402

KEYS = ("primary_rays", "shadow_rays", "reflection_rays", "box_tests", "triangle_tests", "sphere_tests",
        "shading_fetches")


def logical_bytes(c, res_x, res_y):
    """B = 32 N_box + 36 N_tri + 16 N_sph + 16 N_hit + 16 W H."""
    return (32 * c["box_tests"] + 36 * c["triangle_tests"] + 16 * c["sphere_tests"] + 16 * c["shading_fetches"]
            + 16 * res_x * res_y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C3,C5")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "canonical_counts.json"))
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    rt = _rt_pkg.load()
    orc = _rt_pkg.load_oracle()
    ctx = rt.Context()
    res = {}
    if os.path.exists(a.out):
        res = json.load(open(a.out))
    for name in a.configs.split(","):
        fr = rt.make(name)
        W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
        ctx.set_scene(fr.scene)
        _, st = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS))
        gpu = {k: int(getattr(st, k)) for k in KEYS}
        nodes, tris, sphs = ctx.export_bvh()
        b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
        t0 = time.perf_counter()
        # row by row blocks keep the oracle's output buffer small
        cpu = {k: 0 for k in KEYS}
        rows = max(1, (1 << 20) // max(1, W))
        for y0 in range(0, H, rows):
            idx = np.arange(y0 * W, min(H, y0 + rows) * W, dtype=np.int32)
            _, c = b4.render_pixels(idx, threads=a.threads)
            for k in KEYS:
                cpu[k] += int(c[k])
        b4.close()
        tree = hashlib.sha256(nodes.tobytes() + tris.tobytes() + sphs.tobytes()).hexdigest()
        entry = {"config": name, "res": [W, H], "spp": fr.spp, "depth": fr.max_bounces, "counts": cpu,
                 "gpu_counting_launch": gpu, "equal": cpu == gpu,
                 "logical_bytes_per_frame": logical_bytes(cpu, W, H), "tree_sha256": tree,
                 "oracle_seconds": round(time.perf_counter() - t0, 2), "oracle_threads": a.threads}
        res[name] = entry
        print(json.dumps(entry), flush=True)
        if cpu != gpu:
            print(f"MISMATCH {name}: " + ", ".join(f"{k} gpu {gpu[k]} oracle {cpu[k]}" for k in KEYS
                                                  if gpu[k] != cpu[k]), flush=True)
    ctx.close()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
    if not all(v["equal"] for v in res.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
