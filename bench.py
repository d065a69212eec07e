"""bench.py — Mrays/s and ms/frame of the MI355X trace path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
    python bench.py --gpus N --in-process        # one process drives N GPUs (rt_create(N))

One step = one frame of the BASELINE.json metric config (C3: 69,132-tri BVH
scene, 1920x1080, 4 spp, depth 8) rendered through the C-ABI with the scene
already resident in HBM and the frame left in HBM.  With N > 1 ranks the
frame's rows are block-cyclic sharded (band_index = rank) and the shards are
gathered to rank 0 over RCCL and reassembled by a HIP kernel — the fixed
frame is split, so scaling is "strong".  value = rays traced by all ranks
(primary + shadow + reflection, counted on device) / max-over-ranks time.
`--gpus N` without a launcher (no WORLD_SIZE) starts the N ranks itself
(torch.distributed.run, before anything touches a GPU); a world size that
differs from --gpus is an error.

Rank 0 prints ONE JSON line with a roofline object for the trace kernel and
a cpu_baseline measured with the C oracle (single-thread brute force, the
reference's algorithm) on a bounded pixel sample of the same frame.
"""
import argparse
import collections
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Frames in flight need one hardware queue per stream plus RCCL's: HIP's
# default of 4 queues per process serialises a fourth render stream behind
# another (measured on a 1/8 shard: 4 streams 13.7 Grays/s per rank with 4
# queues, 22.7 with 8).  Set before the HIP runtime initialises.
# (--hw-queues N, read here before argparse: experiments with more streams; at most 32 on this pool)
_hwq = 8
for _i, _a in enumerate(sys.argv[:-1]):
    if _a == "--hw-queues":
        _hwq = max(1, min(32, int(sys.argv[_i + 1])))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < _hwq:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_hwq)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before the HIP library: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import _rt_pkg  # noqa: E402

METRIC = "Mrays/sec + ms/frame at 1920x1080, 4spp, depth 8; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"


# Issue peaks for the SQ-counter rooflines (MI355X_MICROARCH.md "Chip-level
# parameters" / "Wave scheduling"): 256 CUs x 4 SIMDs, 2.4 GHz; a wave64 VALU
# instruction occupies its SIMD-32 for 2 cycles; one scalar unit per CU
# issues at most one SALU instruction per cycle.
CLOCK_HZ = 2.4e9
VALU_PEAK = 256 * 4 * CLOCK_HZ / 2 / 1e9  # G wave-instructions/s
SALU_PEAK = 256 * CLOCK_HZ / 1e9          # G instructions/s


def logical_bytes(st, res_x, local_rows):
    """B = 32*N_box + 36*N_tri + 16*N_sph + 16*N_hit + 16*W*H
    (every per-ray node/primitive test priced as if fetched from HBM)."""
    return (32 * st.box_tests + 36 * st.triangle_tests + 16 * st.sphere_tests
            + 16 * st.shading_fetches + 16 * res_x * local_rows)


def canonical_check(config, st, whole_frame):
    """The counting launch's counts against the canonical per-config counts
    committed in profiles/canonical_counts.json (tools/canonical_counts.py: the
    CPU oracle's walk of the same tree).  Whole frames only."""
    p = os.path.join(ROOT, "profiles", "canonical_counts.json")
    if not whole_frame:
        return {"state": "n/a (row band)"}
    if not os.path.exists(p):
        return {"state": "missing"}
    e = json.load(open(p)).get(config)
    if not e or "counts" not in e:  # (C4: only its fetched bytes are pinned — no oracle walk of a 4K frame)
        return {"state": "missing"}
    keys = ("primary_rays", "shadow_rays", "reflection_rays", "box_tests", "triangle_tests", "sphere_tests",
            "shading_fetches")
    got = {k: int(getattr(st, k)) for k in keys}
    ok = all(got[k] == e["counts"][k] for k in keys)
    return {"state": "match" if ok else "mismatch", "committed_logical_bytes": e["logical_bytes_per_frame"],
            **({} if ok else {"got": got, "committed": e["counts"]})}


def lib_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def load_pmc(config, lib_path, bands=1):
    """Per-launch PMC counters of the trace kernel (profiles/pmc_<config>.json,
    or pmc_<config>_b<N>.json for one rank's row band of an N-GPU frame;
    written by tools/pmc_round.sh + tools/pmc_summary.py on the GPU box).  Used
    only when it was measured with the library this run loads (sha256 of the
    .so), so the counters describe the code that ran."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json" if bands <= 1 else f"pmc_{config}_b{bands}.json")
    if not os.path.exists(p):
        return None, "missing"
    try:
        d = json.load(open(p))
    except Exception:
        return None, "unreadable"
    if d.get("lib_sha256") != lib_sha256(lib_path):
        return None, "stale (measured with another build of the library)"
    return d, "fresh"


def roofline(pmc, pmc_state, kernel_name, avg_kernel_s, logical):
    """Roofline object of the trace kernel.  HBM: counter-measured bytes per
    launch (TCC_EA0 read/write requests) over the live kernel time; issue:
    SQ_INSTS_VALU / SQ_INSTS_SALU per launch over the same time against the
    chip's issue rates.  `bound` is the most utilised of the three; the
    §8(d) per-ray byte model is reported as logical_bytes (it counts node and
    triangle re-reads that L2 / Infinity Cache serve, so it exceeds HBM peak)."""
    out = {"kernel": kernel_name, "avg_kernel_ms": avg_kernel_s * 1e3, "pmc": pmc_state,
           "logical_bytes_per_launch": logical, "logical_gbs": logical / avg_kernel_s / 1e9}
    legs = {}
    if pmc:
        hbm = pmc.get("hbm_bytes_per_launch")
        c = pmc.get("counters", {})
        if hbm:
            a = hbm / avg_kernel_s / 1e9
            legs["hbm"] = {"achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS,
                           "read_bytes": pmc.get("read_bytes_per_launch"),
                           "write_bytes": pmc.get("write_bytes_per_launch")}
        if c.get("SQ_INSTS_VALU"):
            a = c["SQ_INSTS_VALU"] / avg_kernel_s / 1e9
            legs["valu_issue"] = {"achieved": a, "peak": VALU_PEAK, "unit": "Gwave-inst/s", "frac": a / VALU_PEAK}
        if c.get("SQ_INSTS_SALU"):
            a = c["SQ_INSTS_SALU"] / avg_kernel_s / 1e9
            legs["salu_issue"] = {"achieved": a, "peak": SALU_PEAK, "unit": "Ginst/s", "frac": a / SALU_PEAK}
        if c.get("SQ_WAVE_CYCLES"):
            tot = c["SQ_WAVE_CYCLES"]
            out["wave_time_split"] = {k: c.get(v, 0.0) / tot for k, v in
                                      (("issuing", "SQ_ACTIVE_INST_ANY"), ("waiting_memory", "SQ_WAIT_ANY"),
                                       ("waiting_issue", "SQ_WAIT_INST_ANY"))}
        out["traffic"] = hbm
    else:
        out["traffic"] = None
    if legs:
        bound = max(legs, key=lambda k: legs[k]["frac"])
        out.update({"bound": bound, **{k: legs[bound][k] for k in ("achieved", "peak", "unit", "frac")}})
        out.update(legs)
    else:  # no counters for this build: the HBM leg cannot be priced
        out.update({"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None})
    return out


L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md "L2 (per XCD)": ~34.5 TB/s aggregate over the 8 XCDs


def fetched_leg(config, avg_kernel_s, rt, fr, whole_frame):
    """The memory side a packet tracer has: the bytes a
    frame's traversal and shading request from the cache hierarchy — scalar
    packet fetches once per wave, per-lane fetches once per lane — counted by
    the RT_FETCH_COUNT measuring build (tools/fetch_bytes.py) and pinned in
    profiles/canonical_counts.json; re-measured here with that build when it
    is present (`state`: match / mismatch), priced against the L2's
    bandwidth.  Whole frames only."""
    if not whole_frame:
        return {"state": "n/a (row band)"}
    p = os.path.join(ROOT, "profiles", "canonical_counts.json")
    e = json.load(open(p)).get(config, {}) if os.path.exists(p) else {}
    committed = e.get("fetched_bytes_per_frame")
    live = None
    variant = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", "fetch", "librt_mi355.so")
    if os.path.exists(variant):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from fetch_bytes import timed_path_fetch  # noqa: E402
        live, _, _ = timed_path_fetch(rt, fr, lib_path=variant)
    b = live if live is not None else committed
    if b is None:
        return {"state": "missing"}
    a = b / avg_kernel_s / 1e9
    return {"bytes_per_launch": b, "achieved": a, "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": a / L2_PEAK_GBS,
            "committed_bytes_per_launch": committed,
            "state": ("match" if live is not None and committed is not None and abs(live - committed) <= 1e-6 * committed
                      else "mismatch" if live is not None and committed is not None
                      else "live (not committed)" if live is not None else "committed (no measuring build)")}


def trace_kernel_name(mode, spp, depth, res_x, local_rows, in_flight=True):
    """The trace kernel instance a frame launches (rtk::launch_render_mega and
    lpt_prepare in csrc/trace.hip / csrc/rt_frame.cpp): the all-packet levels
    kernel for >= 16 spp, otherwise render_kernel<COUNT, SPLIT, DEEP, Q4, W> —
    SPLIT when the frame splits its slowest tiles — shards always (quarter-
    and sixteenth-waves up to 24,000 tiles, sixteenth-waves above), whole
    frames only when no frame of another stream runs beside them (lpt_prepare
    overlapped_frame; `in_flight` False: frames one at a time) — Q4 for 2x2
    spp, W the waves per SIMD (5 for shards of <= 70,000 tiles and deep
    frames, else 6), SAMPLE (the sixth) for the lone-shard instance whose
    one-sample waves trace with the whole wave (csrc/coop.h).  The bench's timed frames are in flight (eight streams):
    whole frames run the non-split instance."""
    if mode == "packet":
        return "render_packet_kernel<false, true>"
    if mode == "wavefront":
        return "wavefront passes (sum)"
    deep = depth > 32  # rtd::kMaxBounces
    if spp >= 16 and not deep:
        fd = 8 if depth <= 8 else 16 if depth <= 16 else 32  # the fold stack's depth bucket
        if spp > 16 and spp != 64:
            return "render_levels_kernel<7, 32, 0>"
        return f"render_levels_kernel<{6 if spp <= 16 else 7}, {fd}, {4 if spp <= 16 else 8}>"
    ppw = 64 // spp
    lg = ppw.bit_length() - 1
    th = 1 << (lg // 2) if ppw & (ppw - 1) == 0 else 1
    tw = ppw // th
    tiles = -(-res_x // tw) * -(-local_rows // th)
    split = not deep and ((16 % spp == 0 and tiles <= 24000) or (4 % spp == 0 and (tiles <= 70000 or not in_flight)))
    # (in flight, shards of more than 24,000 tiles take the 6-wave split instance)
    waves = 5 if deep or (split and tiles <= 70000 and not (in_flight and tiles > 24000)) else 6
    # a lone shard of <= 40,000 tiles at 4 spp: one-sample waves, the SAMPLE instance
    sample = split and not in_flight and spp == 4 and tiles <= 40000
    b = lambda v: "true" if v else "false"  # noqa: E731
    return (f"render_kernel<false, {b(split)}, {b(deep)}, {b(spp == 4 and tw == 4 and th == 4 and not deep)}, "
            f"{waves}, {b(sample)}>")


def host_facts():
    """Host core count and CPU model (BASELINE.md CPU-baseline plan)."""
    model = platform.processor() or ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "affinity_cpus": affinity, "cpu_model": model}


def cpu_baseline(rt, fr, budget_s, ctx):
    """The C oracle (brute force, the reference's algorithm) on seeded random
    pixels of the same frame: 1 thread (the reference is single-threaded
    Mono) for budget_s, then OpenMP over every host core this job is given
    (the affinity mask, capped by OMP_NUM_THREADS: the GPU box grants a
    one-GPU job 16 cores of a larger machine) for budget_s / 3, then the same
    threads with a CPU BVH for budget_s / 3, then with the GPU's own tree
    (bvh_same_tree, rt_export_bvh) for budget_s / 3; plus whole C1 and C2
    frames (median of 5, 1 thread and all threads).  Mrays/s with the same ray
    accounting as the GPU line."""
    orc = _rt_pkg.load_oracle()
    rng = np.random.default_rng(20250101)
    total = fr.plane.ResolutionX * fr.plane.ResolutionY
    rays, secs, pixels = 0, 0.0, 0
    batch = 8
    while secs < budget_s:
        idx = rng.integers(0, total, batch).astype(np.int32)
        t0 = time.perf_counter()
        _, c = orc.render_pixels(fr, idx, threads=1)
        secs += time.perf_counter() - t0
        rays += c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
        pixels += batch
    facts = host_facts()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(facts["affinity_cpus"], omp) if omp else facts["affinity_cpus"])
    mrays, msecs, mpix = 0, 0.0, 0
    while msecs < budget_s / 3:
        idx = rng.integers(0, total, 64 * threads).astype(np.int32)
        t0 = time.perf_counter()
        _, c = orc.render_pixels(fr, idx, threads=threads)
        msecs += time.perf_counter() - t0
        mrays += c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
        mpix += len(idx)
    # the same pixels' closest hits through a CPU BVH (oracle BVH mode, equal
    # answers): the algorithmic part of the GPU's speed-up, separated from
    # the hardware part; tree build outside the timing
    bvh = orc.BvhScene(fr)
    brays, bsecs, bpix = 0, 0.0, 0
    while bsecs < budget_s / 3:
        idx = rng.integers(0, total, 64 * threads).astype(np.int32)
        t0 = time.perf_counter()
        _, c = bvh.render_pixels(idx, threads=threads)
        bsecs += time.perf_counter() - t0
        brays += c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
        bpix += len(idx)
    bvh.close()
    # the GPU's own tree (rt_export_bvh) traversed on the CPU, same threads
    nodes, tris, sphs = ctx.export_bvh()
    b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
    srays, ssecs, spix = 0, 0.0, 0
    while ssecs < budget_s / 3:
        idx = rng.integers(0, total, 64 * threads).astype(np.int32)
        t0 = time.perf_counter()
        _, c = b4.render_pixels(idx, threads=threads)
        ssecs += time.perf_counter() - t0
        srays += c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
        spix += len(idx)
    b4.close()
    # whole frames of the small configs (C1 and C2 in full), the
    # reference's brute force at 1 thread and at the job's threads, median of 5
    full = {}
    for name, reps in (("C1", 5), ("C2", 5)):
        ff = rt.make(name)
        for nt in (1, threads):
            ts, rays_f = [], 0
            for _ in range(reps):
                t0 = time.perf_counter()
                _, c = orc.render(ff, threads=nt)
                ts.append(time.perf_counter() - t0)
                rays_f = c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
            med = float(np.median(ts))
            full[f"{name.lower()}_full" + ("" if nt == 1 else f"_threads_{nt}")] = {
                "mrays_per_s": rays_f / med / 1e6, "ms_per_frame": med * 1e3, "rays_per_frame": rays_f,
                "threads": nt, "runs": reps, "frame": f"{ff.plane.ResolutionX}x{ff.plane.ResolutionY}, "
                                                    f"{ff.spp} spp, depth {ff.max_bounces}"}
    return {
        "value": rays / secs / 1e6,
        "unit": "Mrays/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{pixels} seeded random pixels of {fr.name} ({fr.spp} spp, depth {fr.max_bounces}), "
                  f"{rays} rays in {secs:.1f} s, brute-force C oracle (oracle/rt_oracle.c, gcc -O3 "
                  f"-march=x86-64-v2 -ffp-contract=off), 1 thread (the reference is single-threaded)",
        f"threads_{threads}_value": mrays / msecs / 1e6,
        f"threads_{threads}_sample": f"{mpix} seeded random pixels, {mrays} rays in {msecs:.1f} s",
        # the threads this job may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU pool grants a
        # one-GPU job 16 CPU threads of the host, whatever nproc says)
        "threads_used": threads,
        "threads_why": (f"min(affinity {facts['affinity_cpus']}, OMP_NUM_THREADS {omp}): the pool's CPU share of "
                        f"a one-GPU job" if omp else f"affinity mask {facts['affinity_cpus']}"),
        f"bvh_threads_{threads}_value": brays / bsecs / 1e6,
        f"bvh_threads_{threads}_sample": f"{bpix} seeded random pixels, {brays} rays in {bsecs:.1f} s, the oracle "
                                         f"with a CPU BVH (median split, leaves <= 4; same answers as the scan)",
        "bvh_same_tree": {"mrays_per_s": srays / ssecs / 1e6, "threads": threads,
                          "sample": f"{spix} seeded random pixels, {srays} rays in {ssecs:.1f} s: the GPU's own "
                                    f"4-wide SAH tree (rt_export_bvh) traversed per ray on the CPU like "
                                    f"csrc/traverse.h (near-first closest hits, any-hit shadow rays)"},
        **full,
        **facts,
    }


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """--gpus N without a launcher: run this script as N ranks under
    torch.distributed.run (a child process: nothing here has touched a GPU)
    and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def orbit_cameras(rt, cam0, n, yaw_deg=12.0):
    """n cameras swinging +-yaw_deg about the y axis through the scene centre
    (the origin), looking at it: RayTracingSetup.Update's basis (:175-181) for
    a moving Transform.  Left-handed like Unity: right = up x forward."""
    p0 = np.array(cam0.Position, np.float64)
    r = float(np.linalg.norm(p0))
    out = []
    for k in range(n):
        th = np.radians(yaw_deg) * np.sin(2 * np.pi * k / max(1, n))
        pos = np.array([-r * np.sin(th), p0[1], -r * np.cos(th)])
        fwd = -pos / np.linalg.norm(pos)
        up_w = np.array([0.0, 1.0, 0.0])
        right = np.cross(up_w, fwd)
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        out.append(rt.raytracing.camera_struct(rt.CameraData(tuple(pos), tuple(fwd), tuple(right), tuple(up))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="N>1: check the assembled frame against 1 rank")
    ap.add_argument("--mode", choices=["megakernel", "wavefront", "packet"], default="megakernel")
    ap.add_argument("--streams", type=int, default=8,
                    help="HIP streams the frames are queued on: frames in flight, so one frame's slowest tiles "
                         "overlap the next frames' bulk (1 = one frame at a time; 8 since r07n: the driver's "
                         "command 54.7 Grays/s against 51.8 with 4 streams two deep)")
    ap.add_argument("--gather-frames", type=int, default=0,
                    help="N > 1: frames per RCCL gather (one collective per group of frames; 0 = --streams)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch (rt_render_device_batch: frames of one layout from their own cameras as "
                         "one launch, their tiles under one longest-first order); 0 = 8 for a rank's row band "
                         "(N > 1 or --sim-bands: each band alone is too small to fill the GPU), 1 otherwise")
    ap.add_argument("--pace", type=int, default=1,
                    help="whole frames on one GPU: each frame to the stream with the fewest unfinished frames, at "
                         "most this many a stream (0 = round robin)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="hardware queues per process (GPU_MAX_HW_QUEUES, raised to this before HIP starts)")
    ap.add_argument("--lib", default="", help="experiment: library variant under unity-raytracer_amd/lib/variants/")
    ap.add_argument("--sim-bands", type=int, default=0,
                    help="experiment (one GPU, no gather): render only row band 0 of N, i.e. one rank's share "
                         "of an N-GPU frame")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed path (process group, async gather, reassembly) even at one rank")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo (rehearsal: ranks may share a GPU, "
                         "gather through host memory)")
    ap.add_argument("--in-process", action="store_true",
                    help="one process drives --gpus GPUs through one multi-device context (rt_create(N): row "
                         "bands per GPU, RCCL gather inside the library), as a Unity host would")
    ap.add_argument("--devices", default="",
                    help="--in-process: explicit device list, e.g. 0,0,0 (logical shards on one GPU, peer copies)")
    ap.add_argument("--moving-frames", type=int, default=64,
                    help="N = 1: also time this many frames of an orbiting camera (0 = skip)")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: form the process group, report rank/world on stderr, exit (no GPU work)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.in_process:
        raise SystemExit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.in_process and world != 1:
        raise SystemExit("--in-process runs in one process (no launcher)")
    if not args.in_process and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    gloo = args.dist_backend == "gloo"
    dist_on = world > 1 or args.force_dist
    if args.launch_check:
        if dist_on:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
            # one write per line: both ranks share the launcher's stderr pipe
            os.write(2, (json.dumps({"launch_check": True, "rank": dist.get_rank(),
                                     "world": dist.get_world_size()}) + "\n").encode())
            dist.destroy_process_group()
        else:
            os.write(2, (json.dumps({"launch_check": True, "rank": 0, "world": 1}) + "\n").encode())
        return
    if args.in_process:
        return main_in_process(args)
    ndev = torch.cuda.device_count()
    device = local_rank % ndev if gloo else local_rank
    torch.cuda.set_device(device)
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:  # --force-dist outside a launcher
            os.environ.setdefault("MASTER_PORT", "29531")
        if gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", device))
        world = dist.get_world_size()  # the ranks that actually joined

    rt = _rt_pkg.load()
    fr = rt.make(args.config)
    lib_path = (os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", args.lib, "librt_mi355.so")
                if args.lib else rt.abi.LIB_PATH)
    ctx = rt.Context(lib_path=lib_path if args.lib else None)
    # a created stream, current for the whole run: the null stream's handle is 0,
    # which rt_set_stream reads as "the context's own stream" (non-blocking,
    # unordered with torch's null stream and with RCCL's waits)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_scene(fr.scene)  # rt_set_scene's default: the 4-wide device LBVH (host SAH if too deep)
    bvh_build = {0: "host SAH, 4-wide", 1: "device LBVH, 4-wide"}.get(ctx.scene_info()["build"], "other")
    rx, ry = fr.plane.ResolutionX, fr.plane.ResolutionY
    R = 8
    band_count = world if not args.sim_bands else args.sim_bands
    local_rows = ctx.lib.rt_band_rows_local(ry, rank, band_count, R) if (dist_on or args.sim_bands) else ry
    # Frames rotate over `--streams` HIP streams (more than one = frames in
    # flight).  N > 1: frames are gathered to rank 0 in groups of G
    # (`--gather-frames`, default = streams): each rank's shards of a group
    # sit back to back in one buffer, one RCCL gather per group (the NCCL
    # stream waits for the group's render streams) moves them over xGMI while
    # the other group renders, and rank 0 reassembles the whole group with one
    # HIP launch (bands.assemble_frames: the stack is the shard of one tall
    # image) before the group's buffers are reused.  One collective per G
    # frames keeps rank 0's host cost per frame (a gather call is ~35 us of
    # host time) below a 1/8 shard's frame time.
    nstreams = max(1, args.streams)
    streams = [stream] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    # Batches (a rank's row band, N > 1 or --sim-bands): the frames of a group
    # go as ONE launch (rt_render_device_batch) into the group's buffer, the
    # groups alternate over two streams (two batches in flight); one
    # collective per group as before.
    batch_on = args.batch > 1 or (args.batch == 0 and (dist_on or args.sim_bands) and band_count > 1)
    # (frames per batch = frames per gather group: --gather-frames, else --batch, else 8 — a 1/8 C3 share:
    # 43.3 Grays/s per rank in batches of 8, 33.7 in 4, 30.3 one frame a launch; r07f)
    batch = max(1, min(args.gather_frames or (args.batch if args.batch > 1 else 8), rt.abi.RT_MAX_BATCH)) \
        if batch_on else 1
    # sharded frames travel as float RGB (RT_FLAG_OUT_RGB32F: the Color values
    # bit for bit without the constant alpha, 12 B/px): a quarter less to gather
    ch = 3 if dist_on else 4
    G = batch if batch > 1 else ((args.gather_frames or nstreams) if dist_on else 1)
    ngroups = 2 if dist_on or batch > 1 else max(1, -(-nstreams // G))
    groups = [torch.empty((G, local_rows, rx, ch), dtype=torch.float32, device="cuda") for _ in range(ngroups)]
    nbuf = G * ngroups
    outs = [groups[b // G][b % G] for b in range(nbuf)]
    out = outs[0]
    nbytes = out.numel() * 4
    mode_flags = {"wavefront": rt.abi.RT_FLAG_WAVEFRONT, "packet": rt.abi.RT_FLAG_PACKET}.get(args.mode, 0)
    if dist_on:
        mode_flags |= rt.abi.RT_FLAG_OUT_RGB32F
    params = rt.frame_params(fr, band_index=rank if dist_on else 0, band_count=band_count, band_rows=R,
                             flags=mode_flags)
    span = local_rows * world  # rows of one frame in the tall group image (>= ry)
    if dist_on:
        gath = [torch.empty((world, G * local_rows, rx, ch), dtype=torch.float32, device="cuda")
                for _ in range(ngroups)] if rank == 0 else [None] * ngroups
        gath_lists = [list(g.unbind(0)) for g in gath] if rank == 0 else [None] * ngroups
        images = [torch.empty((G, span, rx, ch), dtype=torch.float32, device="cuda") for _ in range(ngroups)] \
            if rank == 0 else [None] * ngroups
        if gloo:  # host staging buffers for the rehearsal backend
            groups_h = [torch.empty((G * local_rows, rx, ch), dtype=torch.float32) for _ in range(ngroups)]
            gath_h = [torch.empty((world, G * local_rows, rx, ch), dtype=torch.float32) for _ in range(ngroups)] \
                if rank == 0 else [None] * ngroups
            gath_h_lists = [list(g.unbind(0)) for g in gath_h] if rank == 0 else [None] * ngroups
    pending = [None] * ngroups
    freed = [torch.cuda.Event() for _ in range(ngroups)]

    def begin_gather(g):
        """Group g's shards -> rank 0 (RCCL gather over xGMI, async on the
        NCCL stream, which waits for the current stream); the caller made the
        current stream wait for every stream that rendered into the group."""
        src = groups[g].view(G * local_rows, rx, ch)
        if gloo:
            groups_h[g].copy_(src)
            pending[g] = dist.gather(groups_h[g], gath_h_lists[g] if rank == 0 else None, dst=0, async_op=True)
        else:
            pending[g] = dist.gather(src, gath_lists[g] if rank == 0 else None, dst=0, async_op=True)

    def finish_gather(g):
        """Wait for group g's gather (stream-level wait for RCCL) and let rank
        0 put the group's rows back in order with one HIP reassembly launch;
        then the group's buffers are free (event `freed[g]`)."""
        w = pending[g]
        if w is None:
            return
        w.wait()
        pending[g] = None
        if rank == 0:
            if gloo:
                gath[g].copy_(gath_h[g])
            ctx.assemble_bands(gath[g].data_ptr(), rx, G * span, world, R, images[g].data_ptr(),
                               pixel_bytes=4 * ch, sync=False)

    # Frames are enqueued asynchronously (RT_FLAG_ASYNC): the host keeps the
    # stream fed and rt_finish returns the summed counters of the timed frames.
    aparams = rt.frame_params(fr, band_index=params.band_index, band_count=band_count, band_rows=R,
                              flags=mode_flags | rt.abi.RT_FLAG_ASYNC)
    frame_no = [0]
    last_frame = [0]
    cam_s, plane_s = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)

    def close_group(g, used):
        """Gather group g once its `used` frames are enqueued."""
        sb = streams[(used - 1) % nstreams]
        with torch.cuda.stream(sb):
            for k in range(min(used, nstreams) - 1):
                sb.wait_stream(streams[(used - 2 - k) % nstreams])
            begin_gather(g)

    batch_cams = []
    batch_no = [0]
    # The frame queue of whole frames on one GPU (--pace): the next frame goes
    # to the stream with the fewest unfinished frames, at most PACE_DEPTH per
    # stream (the host waits for a slot, as a renderer waits for a free
    # swap-chain image).  Round robin gave every stream the same number of
    # frames although the hardware serves its queues unevenly: in a 20-frame
    # window two streams ended 1.3 ms before the others (r07g kernel trace).
    # Default: eight streams one deep — every queued frame runs, none waits
    # behind another on its stream, so a window's last frames drain together
    # (alternating lines, r07i/r07l/r07m/r07n: the driver's command 49.7 with
    # four streams in rotation, 51.8 four streams two deep, 54.0 four one
    # deep, 54.7 eight one deep; 200 frames 53.3 / 58.2 / 57.5 / 59.4; eight
    # streams two deep 52.6 / 59.3, twelve 50.9 / 57.8)
    pace = args.pace > 0 and not dist_on and batch == 1 and nstreams > 1 and nbuf == nstreams
    PACE_DEPTH = args.pace
    pace_q = [collections.deque() for _ in range(nstreams)]  # per stream: events of its unfinished frames
    pace_wait = [0.0]  # host seconds spent waiting for a slot (not enqueue work)

    def pick_stream():
        tw = None
        while True:
            for q in pace_q:
                while q and q[0].query():
                    q.popleft()
            i = min(range(nstreams), key=lambda k: len(pace_q[k]))
            if len(pace_q[i]) < PACE_DEPTH:
                if tw is not None:
                    pace_wait[0] += time.perf_counter() - tw
                return i
            if tw is None:
                tw = time.perf_counter()

    def flush_batch():
        """The pending frames of the current group as one launch on the
        group's stream (after the group's previous gather is done), then
        the group's gather."""
        if not batch_cams:
            return
        g = batch_no[0] % ngroups
        sb = streams[g % nstreams]
        ctx.set_stream(sb.cuda_stream)
        if dist_on:
            with torch.cuda.stream(sb):  # RCCL's wait targets the current stream
                finish_gather(g)
        ctx.render_device_batch(list(batch_cams), plane_s, aparams, groups[g].data_ptr(), nbytes)
        if dist_on:
            with torch.cuda.stream(sb):
                begin_gather(g)
        batch_cams.clear()
        batch_no[0] += 1

    def step(cam=None):
        if batch > 1:
            last_frame[0] = frame_no[0]
            batch_cams.append(cam or cam_s)
            frame_no[0] += 1
            if len(batch_cams) == G:
                flush_batch()
            return
        f = frame_no[0]
        b = f % nbuf
        g, j = b // G, b % G
        if pace:
            b = pick_stream()  # (one output buffer per stream: nbuf == nstreams here)
        sb = streams[(j if dist_on else b) % nstreams]
        last_frame[0] = f
        ctx.set_stream(sb.cuda_stream)
        if dist_on:
            if j == 0:  # the group's previous gather: done and reassembled, buffers free
                with torch.cuda.stream(sb):  # RCCL's wait targets the current stream
                    finish_gather(g)
                freed[g].record(sb)
            else:
                sb.wait_event(freed[g])
        ctx.render_device(cam or cam_s, plane_s, aparams, outs[b].data_ptr(), nbytes)
        if pace:
            ev = torch.cuda.Event()  # (a fresh one: a slow stream's pending event may be any age)
            ev.record(sb)
            pace_q[b].append(ev)
        if dist_on and j == G - 1:
            close_group(g, G)
        frame_no[0] += 1

    def drain():
        if batch > 1:
            if batch_cams:  # a partial group: its frames as one launch, the next frame starts a fresh group
                frame_no[0] += G - len(batch_cams)
                flush_batch()
            if dist_on:
                for k in range(ngroups):
                    with torch.cuda.stream(stream):
                        ctx.set_stream(stream.cuda_stream)
                        finish_gather(k)
            ctx.set_stream(stream.cuda_stream)
            return
        if dist_on:
            j = frame_no[0] % G
            if j:  # a partial group: gather it as is and start the next frame on a fresh group
                close_group((frame_no[0] % nbuf) // G, j)
                frame_no[0] += G - j
            for k in range(ngroups):
                g = ((frame_no[0] % nbuf) // G + k) % ngroups
                with torch.cuda.stream(stream):
                    ctx.set_stream(stream.cuda_stream)
                    finish_gather(g)
        ctx.set_stream(stream.cuda_stream)

    # counting launch (untimed): algorithmic work of this rank's frame, and
    # the camera samples the Scene.AABB gate rejects before any object test
    cparams = rt.frame_params(fr, band_index=params.band_index, band_count=band_count, band_rows=R,
                              flags=rt.abi.RT_FLAG_COUNT_TESTS | mode_flags)
    cst = ctx.render_device(fr.camera, fr.plane, cparams, out.data_ptr(), nbytes)
    logical = logical_bytes(cst, rx, local_rows)
    canonical = canonical_check(fr.name, cst, band_count == 1)
    scene_misses = int(cst.primary_scene_misses)

    # setup, untimed: one frame on each stream before the W warmup steps.  A
    # stream's first frame allocates its longest-first state in the library
    # (device buffers, the sort's scratch), which blocks the host for
    # milliseconds; with W < --streams that setup would otherwise land in
    # the timed region (measured: 0.29 ms of host stall per timed frame at
    # K = 20, W = 3).
    if batch > 1:  # a batch on each group's stream: the batch slots' longest-first state
        for _ in range(ngroups * G):
            step()
        drain()
    else:
        for sb in streams:
            ctx.set_stream(sb.cuda_stream)
            ctx.render_device(cam_s, plane_s, aparams, out.data_ptr(), nbytes)
    ctx.finish()
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    drain()
    ctx.finish()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pace_wait[0] = 0.0
    for _ in range(args.steps):
        step()
    host_s = time.perf_counter() - t0 - pace_wait[0]  # host time to enqueue the K frames (not the slot waits)
    drain()
    st = ctx.finish()
    ctx.set_stream(stream.cuda_stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    moot = int(st.shadow_rays_moot)  # counted in rays, answered without a traversal
    # device time of the timed frames: HIP events on the streams the trace
    # kernels ran on, from the first timed frame's start to the last one's
    # end (rt_finish) — with frames in flight, the device time per launch of
    # the instance the timed frames run (the roofline's kernel time)
    kernel_ms = st.kernel_ms
    timed_launch = ctx.last_launch()  # the instance and split shape the last timed frame ran (RT_DEBUG_LAST_LAUNCH)
    sky_tiles = int(timed_launch.split("sky=")[1].split()[0]) if "sky=" in timed_launch else 0
    # a lone frame's kernel time (the same frames back to back on one stream,
    # no gather): such frames split their slowest tiles, so this is the split
    # instance — what one synchronous Update() frame costs
    for _ in range(args.steps):
        ctx.render_device(fr.camera, fr.plane, aparams, out.data_ptr(), nbytes)
    lone_kernel_ms = ctx.finish().kernel_ms
    lone_launch = ctx.last_launch()

    # a moving camera (N = 1): every frame from another viewpoint, so the
    # longest-first order always comes from earlier, different frames
    moving = None
    if not dist_on and not args.sim_bands and args.moving_frames > 0:
        cams = orbit_cameras(rt, fr.camera, args.moving_frames)
        for c in cams[:8]:  # warm the orbit's first views
            step(c)
        drain()
        ctx.finish()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for c in cams:
            step(c)
        drain()
        mst = ctx.finish()
        torch.cuda.synchronize()
        mel = time.perf_counter() - t1
        mrays = mst.primary_rays + mst.shadow_rays + mst.reflection_rays
        moving = {"frames": len(cams), "yaw_deg": 12.0, "mrays_per_s": mrays / mel / 1e6,
                  "ms_per_frame": mel / len(cams) * 1e3, "rays_per_frame": mrays // len(cams)}

    # end-to-end rt_render (synchronous, host Color[] output: includes the D2H
    # copy over PCIe, overlapped with the rendering by row slabs), N = 1 only;
    # reported beside `value`, never as it
    e2e_ms = None
    e2e8_ms = None
    d2h_ms = None
    if not dist_on and not args.sim_bands and rank == 0:
        host = np.empty((ry, rx, 4), dtype=np.float32)
        host8 = np.empty((ry, rx, 4), dtype=np.uint8)
        ctx.set_stream(stream.cuda_stream)
        ts, ts8 = [], []
        for _ in range(12):
            t1 = time.perf_counter()
            ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode_flags), out=host)
            ts.append(time.perf_counter() - t1)
        e2e_ms = float(np.median(ts[2:])) * 1e3
        # Color32 (RGBA8) output, the drop-in's 4x-smaller host format
        for _ in range(12):
            t1 = time.perf_counter()
            ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode_flags | rt.abi.RT_FLAG_OUT_RGBA8), out=host8)
            ts8.append(time.perf_counter() - t1)
        e2e8_ms = float(np.median(ts8[2:])) * 1e3
        # the 33 MB device-to-host copy alone into the same pageable buffer
        src = torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda")
        hs = torch.from_numpy(host)
        cs = []
        for _ in range(6):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            hs.copy_(src)
            cs.append(time.perf_counter() - t1)
        d2h_ms = float(np.median(cs[1:])) * 1e3

    if dist_on and args.verify:
        # the assembled frame must be bit-identical to a single-rank frame
        full = torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda")
        if rank == 0:
            ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=mode_flags & ~rt.abi.RT_FLAG_OUT_RGB32F),
                              full.data_ptr(),
                              full.numel() * 4)
            lb = last_frame[0] % nbuf
            last = images[lb // G][lb % G, :ry]
            same = bool(torch.equal(full[..., :ch].contiguous().view(torch.int32), last.view(torch.int32)))
            print(json.dumps({"verify_sharded_equals_single": same}), file=sys.stderr, flush=True)
            if not same:
                ref = full[..., :ch].contiguous().view(torch.int32)
                diag = {"last_frame": last_frame[0], "group": lb // G, "slot": lb % G,
                        "images_equal": [[bool(torch.equal(images[g][k, :ry].view(torch.int32), ref))
                                          for k in range(G)] for g in range(ngroups)]}
                if world == 1:
                    diag["shards_equal"] = [[bool(torch.equal(groups[g][k, :ry].view(torch.int32), ref))
                                             for k in range(G)] for g in range(ngroups)]
                    diag["gathered_equal"] = [[bool(torch.equal(gath[g][0, k * ry:(k + 1) * ry].view(torch.int32),
                                                                ref)) for k in range(G)] for g in range(ngroups)]
                print(json.dumps(diag), file=sys.stderr, flush=True)
                raise SystemExit("sharded frame differs from the single-rank frame")
    if dist_on:
        t = torch.tensor([elapsed, float(rays), kernel_ms, float(scene_misses), float(moot), lone_kernel_ms],
                         dtype=torch.float64, device="cpu" if gloo else "cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        rays = int(t[1])
        kernel_ms_max = float(tmax[2])
        scene_misses = int(t[3])
        moot = int(t[4])
        lone_kernel_ms_max = float(tmax[5])
    else:
        kernel_ms_max = kernel_ms
        lone_kernel_ms_max = lone_kernel_ms

    if rank == 0:
        avg_kernel_s = kernel_ms / args.steps / 1e3  # rank 0's timed frames, HIP events
        pmc, pmc_state = load_pmc(args.config, lib_path, band_count)
        kname = trace_kernel_name(args.mode, fr.spp, fr.max_bounces, rx, local_rows, in_flight=nstreams > 1)
        if batch > 1 and timed_launch.startswith("render_batch_kernel"):
            # one launch renders `batch` frames: per-launch counters are not per-frame figures
            kname = timed_launch.split()[0]
            pmc, pmc_state = None, f"not measured for batch launches ({batch} frames a launch)"
        rays_per_frame = rays // args.steps
        fetched = fetched_leg(args.config, avg_kernel_s, rt, fr,
                              band_count == 1 and batch == 1 and args.mode == "megakernel")
        line = {
            "metric": METRIC,
            "value": rays / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{fr.name}: {fr.scene.triangle_count}-triangle BVH scene (procedural torus-knot "
                            f"stand-in for the ~69k-tri bunny), {rx}x{ry}, {fr.spp} spp, depth {fr.max_bounces}",
                "resolution": f"{rx}x{ry}",
                "spp": fr.spp,
                "depth": fr.max_bounces,
                "triangles": fr.scene.triangle_count,
                "bvh_build": bvh_build,
                "parallelism": f"row-bands x{world}" + ((" + gloo gather (rehearsal)" if gloo else " + RCCL gather")
                                                        if dist_on else ""),
                "rays_per_frame": rays_per_frame,
                # camera samples that end at the Scene.AABB gate (one slab test,
                # Scene.cs:54) and the rays that enter the scene
                "rays_trivial_miss": scene_misses,
                "rays_in_scene": rays_per_frame - scene_misses,
                "mrays_per_s_in_scene": (rays_per_frame - scene_misses) * args.steps / elapsed / 1e6,
                # shadow rays whose answer cannot change the pixel (a light
                # behind the surface): counted above, not traversed
                "shadow_rays_moot": moot // args.steps,
                "mrays_per_s_traversed": (rays - moot) / elapsed / 1e6,
                "frames_in_flight": batch * min(ngroups, nstreams) if batch > 1 else nstreams,
                "frame_queue": f"paced: <= {PACE_DEPTH} unfinished frames a stream, the next to the emptiest" if pace
                else "round robin",
                "timed_launch": timed_launch,
                "lone_launch": lone_launch,
                "frames_per_gather": G if dist_on else None,
                "frames_per_launch": batch,
                # device time per timed frame (HIP events over the timed frames)
                "kernel_ms_per_frame": kernel_ms_max / args.steps,
                # one frame at a time (the split instance of a lone frame)
                "lone_kernel_ms_per_frame": lone_kernel_ms_max / args.steps,
                "lone_kernel": trace_kernel_name(args.mode, fr.spp, fr.max_bounces, rx, local_rows, in_flight=False),
                # primary samples (W*H*spp of the frame, or of this band) per second
                "msamples_per_s": rx * (local_rows if args.sim_bands else ry) * fr.spp * args.steps / elapsed / 1e6,
                "end_to_end_ms_per_frame": e2e_ms,
                "end_to_end_rgba8_ms_per_frame": e2e8_ms,
                "d2h_copy_ms_per_frame": d2h_ms,
                "moving_camera": moving,
                # rank 0's host time per enqueued frame: near ms_per_step means host-bound
                "host_enqueue_ms_per_frame": host_s / args.steps * 1e3,
            },
            "roofline": {**roofline(pmc, pmc_state, kname, avg_kernel_s, logical), "canonical_counts": canonical,
                         # the requested (cache-level) bytes: per-wave packet fetches, per-lane chain fetches
                         "fetched_bytes_per_launch": fetched.get("bytes_per_launch"), "fetched": fetched,
                         # whole frames in flight: the order's sky tail in a second launch per frame
                         # (trace.hip sky_batch_kernel); avg_kernel_ms and the counters cover both
                         **({"with": "sky_batch_batch_kernel" if batch > 1 else
                             f"sky_batch_kernel<{'true' if fr.spp == 4 else 'false'}>",
                             "with_tiles": sky_tiles} if sky_tiles else {})},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(rt, fr, args.cpu_seconds, ctx)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist_on:
        dist.destroy_process_group()


def main_in_process(args):
    """One process, one multi-device context (rt_create(N) / rt_create_devices):
    the library renders row bands on every GPU, gathers them to device 0
    (RCCL send/recv) and reassembles — the path a Unity host takes.  Frames
    rotate over --streams streams of device 0 with RT_FLAG_ASYNC."""
    rt = _rt_pkg.load()
    fr = rt.make(args.config)
    devices = [int(d) for d in args.devices.split(",")] if args.devices else list(range(args.gpus))
    torch.cuda.set_device(devices[0])
    ctx = rt.Context(devices=devices)
    info = ctx.device_info()
    streams = [torch.cuda.Stream() for _ in range(max(1, args.streams))]
    torch.cuda.set_stream(streams[0])
    ctx.set_stream(streams[0].cuda_stream)
    t_scene = time.perf_counter()
    ctx.set_scene(fr.scene)
    scene_s = time.perf_counter() - t_scene
    rx, ry = fr.plane.ResolutionX, fr.plane.ResolutionY
    outs = [torch.empty((ry, rx, 4), dtype=torch.float32, device="cuda") for _ in streams]
    nbytes = outs[0].numel() * 4
    cam_s, plane_s = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
    aparams = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
    cparams = rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS)
    cst = ctx.render_device(cam_s, plane_s, cparams, outs[0].data_ptr(), nbytes)
    frame = [0]

    def step():
        k = frame[0] % len(streams)
        ctx.set_stream(streams[k].cuda_stream)
        ctx.render_device(cam_s, plane_s, aparams, outs[k].data_ptr(), nbytes)
        frame[0] += 1

    for _ in range(len(streams) + args.warmup):
        step()
    ctx.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    host_s = time.perf_counter() - t0
    st = ctx.finish()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    verified = None
    if args.verify:
        single = rt.Context()
        single.set_scene(fr.scene)
        ref = torch.empty_like(outs[0])
        single.render_device(cam_s, plane_s, rt.frame_params(fr), ref.data_ptr(), nbytes)
        ctx.set_stream(streams[0].cuda_stream)
        ctx.render_device(cam_s, plane_s, rt.frame_params(fr), outs[0].data_ptr(), nbytes)
        verified = bool(torch.equal(outs[0].view(torch.int32), ref.view(torch.int32)))
        print(json.dumps({"verify_sharded_equals_single": verified}), file=sys.stderr, flush=True)
        single.close()
        if not verified:
            raise SystemExit("multi-device frame differs from the single-device frame")
    n_gpus = len(set(devices))
    line = {
        "metric": METRIC,
        "value": rays / elapsed / 1e6,
        "unit": "Mrays/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{fr.name}: {fr.scene.triangle_count}-triangle BVH scene, {rx}x{ry}, {fr.spp} spp, "
                        f"depth {fr.max_bounces}",
            "resolution": f"{rx}x{ry}", "spp": fr.spp, "depth": fr.max_bounces,
            "parallelism": f"in-process row-bands x{info['num_devices']} on devices {info['devices']} + "
                           + {0: "no gather", 1: "peer-copy gather", 2: "RCCL gather"}[info["gather"]],
            "rays_per_frame": rays // args.steps,
            "rays_trivial_miss": int(cst.primary_scene_misses),
            "frames_in_flight": len(streams),
            "kernel_ms_per_frame": st.kernel_ms / args.steps,
            "host_enqueue_ms_per_frame": host_s / args.steps * 1e3,
            "set_scene_ms": scene_s * 1e3,
            "verified": verified,
        },
    }
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
