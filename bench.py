"""bench.py — Mrays/s and ms/frame of the MI355X trace path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one frame of the BASELINE.json metric config (C3: 69,132-tri BVH
scene, 1920x1080, 4 spp, depth 8) rendered through the C-ABI with the scene
already resident in HBM and the frame left in HBM.  With N > 1 ranks the
frame's rows are block-cyclic sharded (band_index = rank) and the shards are
gathered to rank 0 over RCCL and reassembled by a HIP kernel — the fixed
frame is split, so scaling is "strong".  value = rays traced by all ranks
(primary + shadow + reflection, counted on device) / max-over-ranks time.

Rank 0 prints ONE JSON line with a roofline object for the trace kernel and
a cpu_baseline measured with the C oracle (single-thread brute force, the
reference's algorithm) on a bounded pixel sample of the same frame.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Frames in flight need one hardware queue per stream plus RCCL's: HIP's
# default of 4 queues per process serialises a fourth render stream behind
# another (measured on a 1/8 shard: 4 streams 13.7 Grays/s per rank with 4
# queues, 22.7 with 8).  Set before the HIP runtime initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before the HIP library: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import _rt_pkg  # noqa: E402

METRIC = "Mrays/sec + ms/frame at 1920x1080, 4spp, depth 8; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"


def algorithmic_bytes(st, res_x, local_rows):
    """B = 32*N_box + 36*N_tri + 16*N_sph + 16*N_hit + 16*W*H."""
    return (32 * st.box_tests + 36 * st.triangle_tests + 16 * st.sphere_tests
            + 16 * st.shading_fetches + 16 * res_x * local_rows)


def cpu_baseline(rt, fr, budget_s):
    """Single-thread brute-force oracle (the reference's algorithm, which is
    single-threaded Mono C#) on seeded random pixels of the same frame,
    until budget_s of CPU time: returns Mrays/s (same ray accounting)."""
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
    # the same code on the host cores the box gives this job (OpenMP over pixels)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
    mrays, msecs = 0, 0.0
    while msecs < budget_s / 3:
        idx = rng.integers(0, total, 64 * threads).astype(np.int32)
        t0 = time.perf_counter()
        _, c = orc.render_pixels(fr, idx, threads=threads)
        msecs += time.perf_counter() - t0
        mrays += c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
    return {
        "value": rays / secs / 1e6,
        "unit": "Mrays/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{pixels} seeded random pixels of {fr.name} ({fr.spp} spp, depth {fr.max_bounces}), "
                  f"{rays} rays in {secs:.1f} s, brute-force C oracle (oracle/rt_oracle.c), 1 thread "
                  f"(the reference is single-threaded)",
        "all_cores_value": mrays / msecs / 1e6,
        "all_cores_threads": threads,
    }


def load_traffic(config):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="N>1: check the assembled frame against 1 rank")
    ap.add_argument("--mode", choices=["megakernel", "wavefront", "packet"], default="megakernel")
    ap.add_argument("--streams", type=int, default=4,
                    help="HIP streams consecutive frames alternate on: frames in flight, so one frame's slowest "
                         "tiles overlap the next frame's bulk (1 = one frame at a time)")
    ap.add_argument("--gather-frames", type=int, default=0,
                    help="N > 1: frames per RCCL gather (one collective per group of frames; 0 = --streams)")
    ap.add_argument("--lib", default="", help="experiment: library variant under unity-raytracer_amd/lib/variants/")
    ap.add_argument("--sim-bands", type=int, default=0,
                    help="experiment (one GPU, no gather): render only row band 0 of N, i.e. one rank's share "
                         "of an N-GPU frame")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed path (process group, async gather, reassembly) even at one rank")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank) or gloo (rehearsal: ranks may share a GPU, "
                         "gather through host memory)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    gloo = args.dist_backend == "gloo"
    dist_on = world > 1 or args.force_dist
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

    rt = _rt_pkg.load()
    fr = rt.make(args.config)
    ctx = rt.Context(lib_path=os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", args.lib, "librt_mi355.so")
                     if args.lib else None)
    # a created stream, current for the whole run: the null stream's handle is 0,
    # which rt_set_stream reads as "the context's own stream" (non-blocking,
    # unordered with torch's null stream and with RCCL's waits)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_scene(fr.scene)
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
    # sharded frames travel as float RGB (RT_FLAG_OUT_RGB32F: the Color values
    # bit for bit without the constant alpha, 12 B/px): a quarter less to gather
    ch = 3 if dist_on else 4
    G = (args.gather_frames or nstreams) if dist_on else 1
    ngroups = 2 if dist_on else max(1, -(-nstreams // G))
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

    def step():
        f = frame_no[0]
        b = f % nbuf
        g, j = b // G, b % G
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
        ctx.render_device(cam_s, plane_s, aparams, outs[b].data_ptr(), nbytes)
        if dist_on and j == G - 1:
            close_group(g, G)
        frame_no[0] += 1

    def drain():
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

    # counting launch (untimed): algorithmic work of this rank's frame
    cparams = rt.frame_params(fr, band_index=params.band_index, band_count=band_count, band_rows=R,
                              flags=rt.abi.RT_FLAG_COUNT_TESTS | mode_flags)
    cst = ctx.render_device(fr.camera, fr.plane, cparams, out.data_ptr(), nbytes)
    bytes_per_launch = algorithmic_bytes(cst, rx, local_rows)

    # setup, untimed: one frame on each stream before the W warmup steps.  A
    # stream's first frame allocates its longest-first state in the library
    # (device buffers, the sort's scratch), which blocks the host for
    # milliseconds; with W < --streams that setup would otherwise land in
    # the timed region (measured: 0.29 ms of host stall per timed frame at
    # K = 20, W = 3).
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
    for _ in range(args.steps):
        step()
    host_s = time.perf_counter() - t0  # host time to enqueue the K frames
    drain()
    st = ctx.finish()
    ctx.set_stream(stream.cuda_stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    # kernel-only device time of this rank's trace launch: the same frames
    # back to back without the gather, HIP events on the context's stream
    for _ in range(args.steps):
        ctx.render_device(fr.camera, fr.plane, aparams, out.data_ptr(), nbytes)
    kernel_ms = ctx.finish().kernel_ms

    # end-to-end rt_render (synchronous, host Color[] output: includes the D2H
    # copy over PCIe), N = 1 only; reported beside `value`, never as it
    e2e_ms = None
    if not dist_on and not args.sim_bands and rank == 0:
        host = np.empty((ry, rx, 4), dtype=np.float32)
        ctx.set_stream(stream.cuda_stream)
        ts = []
        for _ in range(6):
            t1 = time.perf_counter()
            ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=mode_flags), out=host)
            ts.append(time.perf_counter() - t1)
        e2e_ms = float(np.median(ts[1:])) * 1e3

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
        t = torch.tensor([elapsed, float(rays), kernel_ms], dtype=torch.float64,
                         device="cpu" if gloo else "cuda")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        rays = int(t[1])
        kernel_ms_max = float(tmax[2])
    else:
        kernel_ms_max = kernel_ms

    if rank == 0:
        avg_kernel_s = kernel_ms / args.steps / 1e3  # rank 0's own trace kernel, HIP events
        traffic = load_traffic(args.config)
        achieved = bytes_per_launch / avg_kernel_s / 1e9
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
                "parallelism": f"row-bands x{world}" + ((" + gloo gather (rehearsal)" if gloo else " + RCCL gather")
                                                        if dist_on else ""),
                "rays_per_frame": rays // args.steps,
                "frames_in_flight": nstreams,
                "frames_per_gather": G if dist_on else None,
                "kernel_ms_per_frame": kernel_ms_max / args.steps,
                # primary samples (W*H*spp of the frame, or of this band) per second
                "msamples_per_s": rx * (local_rows if args.sim_bands else ry) * fr.spp * args.steps / elapsed / 1e6,
                "end_to_end_ms_per_frame": e2e_ms,
                # rank 0's host time per enqueued frame: near ms_per_step means host-bound
                "host_enqueue_ms_per_frame": host_s / args.steps * 1e3,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": {"megakernel": "render_kernel<false>", "packet": "render_packet_kernel<false,1>"}.get(
                    args.mode, "wavefront passes (sum)"),
                "bytes_per_launch": bytes_per_launch,
                "avg_kernel_ms": avg_kernel_s * 1e3,
                # rocprof-measured HBM bytes (PMC, profiles/pmc_<config>.json) per
                # launch over the same launch time: the bandwidth actually drawn
                "traffic_gbs": (traffic / avg_kernel_s / 1e9) if traffic else None,
                "traffic_frac": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(rt, fr, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
