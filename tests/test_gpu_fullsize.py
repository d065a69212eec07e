"""Full-size, whole-frame parity of the exact paths the bench times
(VERDICT r04 "Next" item 2; SURVEY §8(a) rows A1-A14 at BASELINE sizes).

* The timed path: bench.py's loop — a fresh context, eight HIP streams one
  frame deep (each frame to a stream whose previous frame has ended),
  RT_FLAG_ASYNC frames into device buffers (rt_render_device), enough frames
  that longest-first dispatch runs from a measured order and every stream
  has a frame beside it, so the frames run the in-flight instance
  render_kernel<false, false, false, true, 6, false> (checked through rt_debug_read
  RT_DEBUG_LAST_LAUNCH).  Every pixel of full 1920x1080 C2 and C3 frames must
  equal, bit for bit, the CPU oracle's walk of the same exported 4-wide tree
  (oracle/rt_oracle.c bvh4_query, itself pinned to the brute-force scan of
  Scene.cs:43-122 by tests/test_oracle_bvh4.py and tests/test_gpu_counts.py),
  and the reference's brute force (RayTracingSetup.cs:288-366 over
  Scene.IntersectRay) on seeded pixels; per-frame ray counts equal the
  oracle's.
* A synchronous frame (Unity's Update(), RayTracingSetup.cs:171-199): a lone
  whole frame splits its slowest tiles (render_kernel<false, true, false,
  true, 6>); the same checks.
* C4 (3840x2160, 16 spp) and C5 (250k triangles, 64 spp, depth 16) whole
  frames (render_levels_kernel): every 16th row against the tree walk, plus
  brute force on seeded pixels.
* C4's timed path (bench.py --config C4): eight streams of RT_FLAG_ASYNC
  frames, the levels kernel in flight with its 16-spp sky batches (the
  measured non-sky tiles as stripes, the sky tail in sky_batch_kernel), every
  16th row of every stream's frame against the tree walk, ray counts against
  the counting launch, brute force on 64 seeded pixels.
"""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]

IN_FLIGHT = "render_kernel<false, false, false, true, 6, false>"
LONE_SPLIT = "render_kernel<false, true, false, true, 6, false>"
RAYS = ("primary_rays", "shadow_rays", "reflection_rays")


def _walk(orc, fr, ctx, rows=None):
    """The oracle's walk of the context's exported tree over whole rows
    (all rows, or the given ones): (len(rows), W, 4) float32 and counts."""
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    rows = np.arange(H) if rows is None else np.asarray(rows)
    nodes, tris, sphs = ctx.export_bvh()
    b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
    try:
        out = np.empty((len(rows), W, 4), np.float32)
        counts = {k: 0 for k in RAYS}
        step = max(1, (1 << 19) // W)
        for i in range(0, len(rows), step):
            r = rows[i:i + step]
            idx = (r[:, None] * W + np.arange(W)[None, :]).astype(np.int32).ravel()
            px, c = b4.render_pixels(idx)
            out[i:i + len(r)] = px.reshape(len(r), W, 4)
            for k in RAYS:
                counts[k] += int(c[k])
    finally:
        b4.close()
    return out, counts


def _same_bits(a, b, what):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    assert a.shape == b.shape, what
    diff = a.view(np.uint32) != b.view(np.uint32)
    if diff.any():
        ys, xs = np.nonzero(diff.any(axis=-1))
        err = float(np.nanmax(np.abs(a.astype(np.float64) - b.astype(np.float64))))
        pytest.fail(f"{what}: {len(ys)} pixels differ (first at row {ys[0]}, x {xs[0]}), max |diff| {err}")


def _brute_force(orc, fr, img, n, seed):
    """The reference's algorithm (brute-force scan) on seeded pixels."""
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    idx = np.random.default_rng(seed).choice(W * H, n, replace=False).astype(np.int32)
    ref, _ = orc.render_pixels(fr, idx)
    _same_bits(img.reshape(-1, 4)[idx], ref, f"{fr.name}: brute force on {n} seeded pixels")


@pytest.mark.parametrize("name", ["C3", "C2"])
def test_timed_path_full_frame_equals_oracle(rt, orc, name):
    fr = rt.make(name)
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    ctx = rt.Context()
    streams = [torch.cuda.Stream() for _ in range(8)]
    try:
        ctx.set_stream(streams[0].cuda_stream)
        ctx.set_scene(fr.scene)
        outs = [torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in streams]
        nbytes = outs[0].numel() * 4
        p = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
        cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
        # bench.py: one untimed frame per stream, rt_finish, then the frames
        for k, s in enumerate(streams):
            ctx.set_stream(s.cuda_stream)
            ctx.render_device(cam, pl, p, outs[k].data_ptr(), nbytes)
        ctx.finish()
        torch.cuda.synchronize()
        frames, launches, used = 48, [], [0] * len(streams)
        done = [None] * len(streams)  # per stream: the event of its unfinished frame (bench.py's paced queue)
        for f in range(frames):
            while True:  # a stream whose previous frame has ended (each stream's order measured by its setup frame)
                free = [k for k in range(len(streams)) if done[k] is None or done[k].query()]
                if free:
                    break
            k = min(free, key=lambda j: used[j])
            used[k] += 1
            ctx.set_stream(streams[k].cuda_stream)
            ctx.render_device(cam, pl, p, outs[k].data_ptr(), nbytes)
            done[k] = torch.cuda.Event()
            done[k].record(streams[k])
            launches.append(ctx.last_launch())
        st = ctx.finish()
        torch.cuda.synchronize()
        # every frame with another stream's frame pending beside it runs the in-flight instance
        assert all(l.startswith(IN_FLIGHT) for l in launches[1:]), launches[:6]
        # ... and renders its measured sky tail in sky_batch_kernel (C3's knot
        # and C2's open room both fill the centre of the view: 77,616 of the
        # 129,600 tiles miss the scene box)
        sky = [int(l.split("sky=")[1].split()[0]) for l in launches[1:]]
        assert all(s > 0 for s in sky), launches[:6]
        imgs = [o.cpu().numpy() for o in outs]
        ctx.set_stream(None)
        ref, counts = _walk(orc, fr, ctx)
    finally:
        ctx.close()
    for k in range(1, len(imgs)):
        _same_bits(imgs[k], imgs[0], f"{name}: stream {k} vs stream 0")
    _same_bits(imgs[0], ref, f"{name}: timed path vs the oracle's walk of the same tree, whole frame")
    assert tuple(getattr(st, k) // frames for k in RAYS) == tuple(counts[k] for k in RAYS)
    assert all(getattr(st, k) % frames == 0 for k in RAYS)
    _brute_force(orc, fr, imgs[0], 3000 if name == "C3" else 6000, seed=11)


@pytest.mark.parametrize("name", ["C3", "C2"])
def test_synchronous_full_frame_equals_oracle(rt, orc, name):
    """One frame at a time (Update()): the lone frame's split instance."""
    fr = rt.make(name)
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    ctx = rt.Context()
    try:
        ctx.set_scene(fr.scene)
        out = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
        for _ in range(3):  # the first frame measures the tile order; the next ones split by it
            st = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr), out.data_ptr(), out.numel() * 4)
        launch = ctx.last_launch()
        assert launch.startswith(LONE_SPLIT) and "split16=0" not in launch, launch
        img = out.cpu().numpy()
        ref, counts = _walk(orc, fr, ctx)
    finally:
        ctx.close()
    _same_bits(img, ref, f"{name}: synchronous frame vs the oracle's walk, whole frame")
    assert tuple(getattr(st, k) for k in RAYS) == tuple(counts[k] for k in RAYS)
    _brute_force(orc, fr, img, 2000, seed=12)


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_levels_full_frame_every_16th_row(rt, orc, name):
    fr = rt.make(name)
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    ctx = rt.Context()
    try:
        ctx.set_scene(fr.scene)
        out = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
        st = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr), out.data_ptr(), out.numel() * 4)
        assert ctx.last_launch().startswith("render_levels_kernel<"), ctx.last_launch()
        img = out.cpu().numpy()
        rows = np.arange(0, H, 16)
        ref, _ = _walk(orc, fr, ctx, rows)
    finally:
        ctx.close()
    _same_bits(img[rows], ref, f"{name}: every 16th row vs the oracle's walk")
    assert st.primary_rays == W * H * fr.spp
    assert np.isfinite(img).all()
    _brute_force(orc, fr, img, 64, seed=13)


def test_c4_timed_path_in_flight_every_16th_row(rt, orc):
    """bench.py --config C4's timed frames: the levels instance in flight with
    its 16-spp sky batches (RT_DEBUG_LAST_LAUNCH sky > 0)."""
    fr = rt.make("C4")
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    ctx = rt.Context()
    streams = [torch.cuda.Stream() for _ in range(8)]  # bench.py's eight streams (one frame each here)
    try:
        ctx.set_stream(streams[0].cuda_stream)
        ctx.set_scene(fr.scene)
        outs = [torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda") for _ in streams]
        nbytes = outs[0].numel() * 4
        # the counting launch (per-lane traversal, the canonical counts' path)
        cst = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS),
                                outs[0].data_ptr(), nbytes)
        p = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
        cam, pl = rt.raytracing.camera_struct(fr.camera), rt.raytracing.plane_struct(fr.plane)
        for k, s in enumerate(streams):  # bench.py's setup: one untimed frame per stream
            ctx.set_stream(s.cuda_stream)
            ctx.render_device(cam, pl, p, outs[k].data_ptr(), nbytes)
        ctx.finish()
        torch.cuda.synchronize()
        for o in outs:
            o.fill_(float("nan"))
        frames, launches = 8, []
        for f in range(frames):
            k = f % len(streams)
            ctx.set_stream(streams[k].cuda_stream)
            ctx.render_device(cam, pl, p, outs[k].data_ptr(), nbytes)
            launches.append(ctx.last_launch())
        st = ctx.finish()
        torch.cuda.synchronize()
        assert all(l.startswith("render_levels_kernel<6, 8, 4>") for l in launches), launches[:2]
        sky = [int(l.split("sky=")[1].split()[0]) for l in launches[1:]]
        assert all(s > 0 for s in sky), launches[:3]
        rows = np.arange(0, H, 16)
        imgs = [o[rows].cpu().numpy() for o in outs]
        full0 = outs[0].cpu().numpy()
        ctx.set_stream(None)
        ref, _ = _walk(orc, fr, ctx, rows)
    finally:
        ctx.close()
    for k in range(len(imgs)):
        _same_bits(imgs[k], ref, f"C4 in flight, stream {k}: every 16th row vs the oracle's walk")
    assert st.primary_rays == frames * W * H * fr.spp
    assert tuple(getattr(st, k) for k in RAYS) == tuple(frames * getattr(cst, k) for k in RAYS)
    assert np.isfinite(full0).all()
    _brute_force(orc, fr, full0, 64, seed=14)
