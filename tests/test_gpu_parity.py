"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar: max |gpu - oracle| <= 1e-4 per RGB channel in Color units (north_star);
the arithmetic is the reference's float32 op order on both sides, so the
observed error is normally exactly 0.  Ray counts (primary / shadow /
reflection) must match the oracle exactly — they are integer decisions.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4  # per RGB channel, Color units (Rgb.Color = Value / 255)


def _render(ctx, rt, fr, build=0, **kw):
    ctx.set_scene(fr.scene, build)
    img, st = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, **kw))
    return img, st


def _check(img, ref, st, counts, name):
    assert img.shape == ref.shape
    err = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    assert np.isfinite(img).all() == np.isfinite(ref).all()
    mx = float(np.nanmax(err)) if err.size else 0.0
    assert mx <= TOL, f"{name}: max err {mx} at {np.unravel_index(np.nanargmax(err), err.shape)}"
    got = (st.primary_rays, st.shadow_rays, st.reflection_rays)
    want = (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"])
    assert got == want, f"{name}: ray counts {got} != oracle {want}"


# name -> (rt_render_params.flags, BVH builder: 0 host SAH, 1 GPU LBVH 4-wide, 2 GPU LBVH 2-wide)
MODES = {"megakernel": (0, 0), "megakernel_count": (1, 0), "wavefront": (2, 0), "packet": (4, 0), "lbvh": (0, 1),
         "lbvh_wavefront": (2, 1),
         "lbvh_packet": (4, 1), "lbvh2": (0, 2)}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name,res,spp", [
    ("demo", None, 1),
    ("C1", None, 1),
    ("C2", (192, 108), 4),
    ("C2", (64, 36), 9),
    ("C3", (96, 54), 4),
    ("C5", (48, 27), 4),
])
def test_frame_vs_oracle(gpu_ctx, rt, orc, name, res, spp, mode):
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=spp)
    flags, build = MODES[mode]
    img, st = _render(gpu_ctx, rt, fr, build=build, flags=flags)
    ref, counts = orc.render(fr)
    _check(img, ref, st, counts, f"{name}/{mode}")


@pytest.mark.parametrize("name,res,spp", [("C3", (48, 27), 16), ("C2", (40, 24), 64), ("C5", (24, 14), 16),
                                          ("C3", (26, 15), 25), ("C2", (22, 13), 36), ("C5", (14, 9), 49),
                                          ("C3", (20, 11), 64)])
def test_levels_kernel_vs_oracle(gpu_ctx, rt, orc, name, res, spp):
    """>= 16 spp frames take the level-synchronous all-packet megakernel
    (render_levels_kernel): whole frames against the oracle, mirror chains
    and their shadow rays included."""
    fr = rt.make(name).with_resolution(*res).with_(spp=spp)
    img, st = _render(gpu_ctx, rt, fr)
    ref, counts = orc.render(fr)
    _check(img, ref, st, counts, f"{name}/levels/{spp}spp")


def test_levels_kernel_bit_identical_to_other_paths(gpu_ctx, rt):
    """The levels kernel, the level-synchronous packet kernel (per-lane deep
    levels) and the wavefront path give the same bits and ray counts."""
    fr = rt.make("C3").with_resolution(480, 270).with_(spp=16)
    a, sa = _render(gpu_ctx, rt, fr, flags=0)
    for flags in (2, 4):
        b, sb = _render(gpu_ctx, rt, fr, flags=flags)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), flags
        assert (sa.primary_rays, sa.shadow_rays, sa.reflection_rays) == (sb.primary_rays, sb.shadow_rays,
                                                                         sb.reflection_rays), flags


def test_modes_bit_identical_full_c3(gpu_ctx, rt):
    """Megakernel, wavefront and packet frames are bit-identical at full C3
    size, and so are their ray counts."""
    fr = rt.make("C3")
    a, sa = _render(gpu_ctx, rt, fr, flags=0)
    for flags in (2, 4):
        b, sb = _render(gpu_ctx, rt, fr, flags=flags)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), flags
        assert (sa.primary_rays, sa.shadow_rays, sa.reflection_rays) == (sb.primary_rays, sb.shadow_rays,
                                                                         sb.reflection_rays), flags


@pytest.mark.parametrize("name,res,spp", [("C3", (96, 54), 4), ("C2", (96, 54), 4), ("C5", (48, 27), 16)])
def test_moot_shadow_rays_are_invisible(gpu_ctx, rt, orc, name, res, spp):
    """Shadow rays whose answer cannot change the pixel (shade.h same_bits:
    the light's unoccluded term leaves the colour's bits unchanged) are not
    traversed by the packet paths: they are still counted in shadow_rays (the
    oracle's count), reported in shadow_rays_moot, and the frame equals the
    oracle's and the counting launch's, which traces every ray per lane."""
    fr = rt.make(name).with_resolution(*res).with_(spp=spp)
    img, st = _render(gpu_ctx, rt, fr)
    ref, counts = orc.render(fr)
    _check(img, ref, st, counts, name)
    assert 0 < st.shadow_rays_moot < st.shadow_rays
    cimg, cst = _render(gpu_ctx, rt, fr, flags=1)
    assert cst.shadow_rays_moot == 0
    assert np.array_equal(img.view(np.uint32), cimg.view(np.uint32))


def test_goldens(gpu_ctx, rt):
    """Committed fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "frames.npz"))
    for name in ("demo", "C1"):
        fr = rt.make(name)
        img, st = _render(gpu_ctx, rt, fr)
        ref = g[name]
        assert float(np.max(np.abs(img[..., :3] - ref))) <= TOL
        assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == tuple(g[name + "_counts"])


@pytest.mark.parametrize("name,npix", [("C2", 2000), ("C3", 400), ("C4", 150), ("C5", 120)])
def test_full_size_sampled_pixels(gpu_ctx, rt, orc, name, npix):
    """BASELINE configs at full size (C2/C3 1080p 4 spp depth 8, C4 4K 16 spp
    depth 8, C5 1080p 64 spp depth 16): the GPU frame against the oracle on
    seeded pixels (pixels are independent, RayTracingSetup.cs:288-301), plus
    the full-frame primary ray count."""
    fr = rt.make(name)
    img, st = _render(gpu_ctx, rt, fr)
    rng = np.random.default_rng(7)
    W, H = fr.plane.ResolutionX, fr.plane.ResolutionY
    idx = rng.choice(W * H, npix, replace=False).astype(np.int32)
    ref, _ = orc.render_pixels(fr, idx)
    got = img.reshape(-1, 4)[idx]
    assert float(np.max(np.abs(got - ref))) <= TOL
    assert st.primary_rays == W * H * fr.spp
    assert np.isfinite(img).all()


def test_intersect_rays_exact(gpu_ctx, rt, orc):
    """Scene.IntersectRay batch query: type, index, mesh index and distance
    equal the brute-force oracle exactly, incl. rays leaving surfaces."""
    for name in ("demo", "C2", "C3", "C5"):
        fr = rt.make(name)
        gpu_ctx.set_scene(fr.scene)
        rng = np.random.default_rng(11)
        n = 4000 if name != "C5" else 1500
        o = rng.uniform(-1.2, 1.2, (n, 3)).astype(np.float32)
        if name == "demo":
            o *= 30
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        d[: n // 10, 0] = 0.0  # axis-parallel components (rcp = +-inf)
        rays = np.concatenate([o, d.astype(np.float32)], 1)
        hits = gpu_ctx.intersect_rays(rays)
        ref = orc.intersect(fr.scene, rays)
        # type, index and ObjectId.MeshIndex exactly, including the stale mesh
        # index the reference leaves when a sphere or loose triangle wins after
        # a mesh triangle (Scene.cs:76-79 set it, :94-97 / :109-112 keep it)
        for f in ("type", "index", "mesh_index"):
            assert np.array_equal(hits[f], ref[f]), (name, f)
        if name in ("C3", "C5"):
            stale = (ref["type"] != 3) & (ref["mesh_index"] >= 0)
            assert stale.any(), name  # the case is exercised
        assert np.array_equal(hits["distance"].view(np.uint32), ref["distance"].view(np.uint32)), name


def test_determinism_and_bands(gpu_ctx, rt):
    """Two renders are bit-identical; row shards reassembled equal the full frame."""
    import torch
    fr = rt.make("C2").with_resolution(200, 123)
    a, _ = _render(gpu_ctx, rt, fr)
    b, _ = _render(gpu_ctx, rt, fr)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for bands in (2, 3, 8):
        rows = gpu_ctx.lib.rt_band_rows_local(fr.plane.ResolutionY, 0, bands, 8)
        parts = []
        for k in range(bands):
            img, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, band_index=k, band_count=bands))
            assert img.shape[0] == rows
            parts.append(img)
        gathered = torch.from_numpy(np.stack(parts)).cuda()
        full = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.assemble_bands(gathered.data_ptr(), fr.plane.ResolutionX, fr.plane.ResolutionY, bands, 8,
                               full.data_ptr())
        assert np.array_equal(full.cpu().numpy().view(np.uint32), a.view(np.uint32)), bands


def test_edge_cases(gpu_ctx, rt, orc):
    S = rt.Scene
    fr0 = rt.make("C1").with_resolution(32, 24)
    # empty scene: everything is background (Shade :310-311)
    empty = fr0.with_(scene=S(), background=(0.25, 0.5, 1.0, 1.0))
    img, st = _render(gpu_ctx, rt, empty)
    assert np.allclose(img[..., :3], np.array([0.25, 0.5, 1.0], np.float32) * np.float32(255) / np.float32(255))
    assert st.shadow_rays == 0
    # spheres only / loose triangles only / one mesh only
    c1 = fr0.scene
    only_sph = S()
    only_sph.SphereData = c1.SphereData
    only_sph.PointLights = c1.PointLights
    only_sph.AmbientLight = c1.AmbientLight
    only_tri = S()
    only_tri.TriangleData = c1.TriangleData
    only_tri.PointLights = c1.PointLights
    for sc in (only_sph, only_tri):
        f = fr0.with_(scene=sc)
        img, st = _render(gpu_ctx, rt, f)
        ref, counts = orc.render(f)
        _check(img, ref, st, counts, "edge")
    # no lights, negative / zero bounces, zero resolution
    for kw in (dict(max_bounces=0), dict(max_bounces=-1)):
        f = fr0.with_(**kw)
        img, st = _render(gpu_ctx, rt, f)
        ref, counts = orc.render(f)
        _check(img, ref, st, counts, "bounces")
    f = fr0.with_resolution(0, 0)
    img, st = _render(gpu_ctx, rt, f)
    assert img.size == 0 and st.primary_rays == 0


def test_errors(gpu_ctx, rt):
    fr = rt.make("C1").with_resolution(8, 8)
    gpu_ctx.set_scene(fr.scene)
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, spp=2))
    assert e.value.status == rt.abi.RT_E_INVALID
    with pytest.raises(rt.RtError) as e:
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, band_index=3, band_count=2))
    assert e.value.status == rt.abi.RT_E_INVALID
    fresh = rt.Context()
    with pytest.raises(rt.RtError) as e:
        fresh.render(fr.camera, fr.plane, rt.frame_params(fr))
    assert e.value.status == rt.abi.RT_E_STATE
    fresh.close()


def test_cpp_host_mirror_demo(tmp_path):
    """The C++ host mirror (unity-raytracer_amd/host/RayTracer.hpp) renders the
    reference demo scene through the C-ABI in a process without torch; its
    PixelColors equal the committed golden frame."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "unity-raytracer_amd", "lib", "cast_pixel_rays")
    out = tmp_path / "demo.f32"
    r = subprocess.run([exe, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = np.fromfile(out, np.float32).reshape(50, 50, 4)
    g = np.load(os.path.join(root, "tests", "golden", "frames.npz"))
    assert np.array_equal(img[..., :3].view(np.uint32), g["demo"].view(np.uint32))
    assert np.all(img[..., 3] == 1.0)


def test_async_frames(gpu_ctx, rt):
    """RT_FLAG_ASYNC frames: same image as a synchronous frame, and rt_finish
    returns the counters of all of them; a synchronous frame in between
    settles the pending ones without losing their counts."""
    import torch
    fr = rt.make("C2").with_resolution(160, 90)
    gpu_ctx.set_scene(fr.scene)
    ref, sr = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    out = torch.empty((90, 160, 4), dtype=torch.float32, device="cuda")
    gpu_ctx.finish()
    k = 5
    for _ in range(k):
        st = gpu_ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC),
                                   out.data_ptr(), out.numel() * 4)
        assert st.primary_rays == 0  # zeroed: counts come from rt_finish
    tot = gpu_ctx.finish()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert (tot.primary_rays, tot.shadow_rays, tot.reflection_rays) == (k * sr.primary_rays, k * sr.shadow_rays,
                                                                        k * sr.reflection_rays)
    assert tot.kernel_ms > 0.0
    # async, then sync, then finish: the async frame is still reported
    gpu_ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC), out.data_ptr(),
                          out.numel() * 4)
    gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    tot = gpu_ctx.finish()
    assert tot.primary_rays == sr.primary_rays
    with pytest.raises(rt.RtError):
        gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC))


def test_longest_first_order_is_invisible(gpu_ctx, rt):
    """Synchronous frames after the first dispatch their tiles longest-first
    (previous frame's costs); the frames stay bit-identical to row-major ones,
    also when the layout or the scene changes in between."""
    fr = rt.make("C3").with_resolution(320, 180)
    gpu_ctx.set_scene(fr.scene)
    row, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER))
    for _ in range(6):  # crosses a re-sort period
        img, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
        assert np.array_equal(img.view(np.uint32), row.view(np.uint32))
    small = fr.with_resolution(64, 48)
    a, _ = gpu_ctx.render(small.camera, small.plane, rt.frame_params(small))
    b, _ = gpu_ctx.render(small.camera, small.plane, rt.frame_params(small, flags=rt.abi.RT_FLAG_ROW_ORDER))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    fr2 = rt.make("C2").with_resolution(320, 180)
    gpu_ctx.set_scene(fr2.scene)
    for _ in range(3):
        c, _ = gpu_ctx.render(fr2.camera, fr2.plane, rt.frame_params(fr2))
    d, _ = gpu_ctx.render(fr2.camera, fr2.plane, rt.frame_params(fr2, flags=rt.abi.RT_FLAG_ROW_ORDER))
    assert np.array_equal(c.view(np.uint32), d.view(np.uint32))


def test_split_slowest_tiles_is_invisible(gpu_ctx, rt):
    """Small frames (<= 24,000 tiles) run their slowest tiles, as measured by
    the previous re-sort, as four quarter-waves (the slowest 1/2048 — in
    synchronous frames as 64 one-sample waves at 4 spp, whose pixel sums meet
    through write-through stores and an arrival count): same bits and same ray
    counts as row-major whole-tile frames, for a whole frame and for a row
    shard."""
    fr = rt.make("C3").with_resolution(640, 360)
    gpu_ctx.set_scene(fr.scene)
    for kw in ({}, dict(band_index=1, band_count=3, band_rows=8)):
        row, sr = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
        for _ in range(3):  # the first frame measures and sorts; later ones split
            img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, **kw))
            assert np.array_equal(img.view(np.uint32), row.view(np.uint32)), kw
            assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (sr.primary_rays, sr.shadow_rays,
                                                                             sr.reflection_rays), kw
            # shadow_rays_moot counts the moot rays a frame did not traverse:
            # the split tiles' per-lane mirror chains skip theirs, whole tiles'
            # per-lane chains trace them (include/rt_mi355.h rt_stats), so a
            # split frame may skip more — never fewer, never more than exist
            assert sr.shadow_rays_moot <= st.shadow_rays_moot <= st.shadow_rays, kw


@pytest.mark.parametrize("res,spp", [((480, 270), 4), ((1920, 1080), 4), ((480, 270), 16)])
def test_sky_batches_render_tiles_that_stopped_being_sky(gpu_ctx, rt, res, spp):
    """Whole frames in flight (another stream's frame beside them) take the
    last measured order's sky tail kSkyBatch tiles a wave (trace.hip
    sky_batch_kernel, RT_DEBUG_LAST_LAUNCH "sky=N"; lone frames and frames of
    <= 24,000 tiles like 480x270 do not; at 16 spp the levels
    kernel's frames of any size do, its positions then the non-sky tiles).  After
    the camera moves the order is stale until the next re-sort: tiles of that
    tail now show the knot and are rendered in full.  Frames equal row-major
    frames bit for bit, with the same ray counts, before and after the move."""
    import torch
    fr = rt.make("C3").with_resolution(*res).with_(spp=spp)
    ctx = rt.Context()  # its own (stream, slab) longest-first slots
    ctx.set_scene(fr.scene)
    c = fr.camera
    moved = rt.CameraData(tuple(float(a + 1.5 * b) for a, b in zip(c.Position, c.Right)), c.Forward, c.Right, c.Up)
    prow = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER)
    row, sr = ctx.render(c, fr.plane, prow)
    row2, sr2 = ctx.render(moved, fr.plane, prow)
    assert not np.array_equal(row2.view(np.uint32), row.view(np.uint32))
    H, W = fr.plane.ResolutionY, fr.plane.ResolutionX
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    pa = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC)
    rays = lambda s: (s.primary_rays, s.shadow_rays, s.reflection_rays)  # noqa: E731

    def pair(cam0):  # a static-camera frame on stream 1, then the frame under test on stream 0 beside it
        for k, cam in ((1, c), (0, cam0)):
            ctx.set_stream(streams[k].cuda_stream)
            ctx.render_device(cam, fr.plane, pa, outs[k].data_ptr(), outs[k].numel() * 4)
        launch = ctx.last_launch()
        st = ctx.finish()
        torch.cuda.synchronize()
        return launch, st, [o.cpu().numpy() for o in outs]

    try:
        for k in range(3):  # frame 0 of each stream measures and sorts; later frames take batches
            launch, st, img = pair(c)
            for i in range(2):
                assert np.array_equal(img[i].view(np.uint32), row.view(np.uint32)), (k, i)
            assert rays(st) == tuple(2 * v for v in rays(sr)), k
        whole = spp == 16 or (res[0] // 4) * (res[1] // 4) > 24000  # rt_frame.cpp kSkyMinTiles
        assert (int(launch.split("sky=")[1].split()[0]) > 0) == whole, launch
        launch, st, img = pair(moved)  # the same (now stale) order, each stream's frame 3 of 32
        assert (int(launch.split("sky=")[1].split()[0]) > 0) == whole, launch
        assert np.array_equal(img[1].view(np.uint32), row.view(np.uint32))
        assert np.array_equal(img[0].view(np.uint32), row2.view(np.uint32))
        assert rays(st) == tuple(a + b for a, b in zip(rays(sr), rays(sr2)))
        # the camera turned away from the scene: every tile is sky; after the
        # re-sort (each stream's frame 32, rt_frame.cpp kLptPeriod) the whole
        # order is the sky tail
        away = rt.CameraData(c.Position, tuple(-v for v in c.Forward), tuple(-v for v in c.Right), c.Up)
        row3, sr3 = ctx.render(away, fr.plane, prow)
        for k in range(30):
            launch, st, img = pair(away)
            assert np.array_equal(img[0].view(np.uint32), row3.view(np.uint32)), k
            assert rays(st) == tuple(a + b for a, b in zip(rays(sr), rays(sr3))), k
        if whole:  # all but one tile (render_kernel keeps a wave)
            assert int(launch.split("sky=")[1].split()[0]) == int(launch.split("tiles=")[1].split()[0]) - 1, launch
        # a lone frame takes no batches
        ctx.set_stream(None)
        ctx.render(c, fr.plane, rt.frame_params(fr))
        assert "sky=0" in ctx.last_launch(), ctx.last_launch()
    finally:
        ctx.set_stream(None)
        ctx.close()


def test_sky_count_waits_only_for_frames_that_use_it(gpu_ctx, rt):
    """A longest-first slot's first sort makes the host wait for its sky-tail
    count only when a frame like it takes sky batches (frames in flight of more
    than 24,000 tiles, rt_frame.cpp sky_tail_usable).  RT_FLAG_ASYNC frames that
    alternate two layouts on one stream re-sort at every layout change and are
    lone frames: no wait (RT_DEBUG_LAST_LAUNCH sky_waits), same bits as
    row-major frames.  Whole frames in flight on two streams do wait, once per
    slot."""
    import torch
    base = rt.make("C3")
    frs = [base.with_resolution(960, 540), base.with_resolution(1920, 1080)]
    ctx = rt.Context()
    ctx.set_scene(base.scene)
    waits = lambda: int(ctx.last_launch().split("sky_waits=")[1].split()[0])  # noqa: E731
    try:
        rows = [ctx.render(f.camera, f.plane, rt.frame_params(f, flags=rt.abi.RT_FLAG_ROW_ORDER))[0] for f in frs]
        outs = [torch.empty(r.shape, dtype=torch.float32, device="cuda") for r in rows]
        s = torch.cuda.Stream()
        ctx.set_stream(s.cuda_stream)
        for k in range(7):
            i = k % 2
            f = frs[i]
            ctx.render_device(f.camera, f.plane, rt.frame_params(f, flags=rt.abi.RT_FLAG_ASYNC), outs[i].data_ptr(),
                              outs[i].numel() * 4)
            assert waits() == 0, (k, ctx.last_launch())
            ctx.finish()
            torch.cuda.synchronize()
            assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), rows[i].view(np.uint32)), k
        # whole 1080p frames in flight: the first sort of each stream's slot waits once
        streams = [s, torch.cuda.Stream()]
        f = frs[1]
        for k in range(6):
            ctx.set_stream(streams[k % 2].cuda_stream)
            ctx.render_device(f.camera, f.plane, rt.frame_params(f, flags=rt.abi.RT_FLAG_ASYNC), outs[1].data_ptr(),
                              outs[1].numel() * 4)
        ctx.finish()
        torch.cuda.synchronize()
        assert 1 <= waits() <= 2, ctx.last_launch()
    finally:
        ctx.set_stream(None)
        ctx.close()


@pytest.mark.parametrize("name,res,band", [("C3", None, (5, 8)), ("C3", None, (0, 8)), ("C3", (480, 270), None),
                                           ("C2", None, (3, 8)), ("C5", (960, 540), (1, 4))])
def test_batches_equal_single_frames(gpu_ctx, rt, name, res, band):
    """rt_render_device_batch: frames of one layout from their own cameras as
    one launch (trace.hip render_batch_kernel; the batch's tiles under one
    longest-first order, its sky tail in sky_batch_batch_kernel) — every frame
    bit-identical to the row-major single frame of its camera, ray counts the
    sum.  Two batches in flight on two streams, then lone batches; the cameras
    change between batches, so a batch's sky tail (measured on other cameras)
    holds tiles that are no longer sky (rendered by the out-of-line per-lane
    path) and its splits fall on other tiles."""
    import torch
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=4)
    ctx = rt.Context()
    ctx.set_scene(fr.scene)
    kw = dict(band_index=band[0], band_count=band[1], band_rows=8) if band else {}
    c = fr.camera
    cams = [c] + [rt.CameraData(tuple(float(a + k * 0.35 * b) for a, b in zip(c.Position, c.Right)), c.Forward, c.Right,
                                c.Up) for k in (1, 2, -1)]
    prow = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw)
    refs, rst = [], []
    for cam in cams:
        img, st = ctx.render(cam, fr.plane, prow)
        refs.append(img)
        rst.append((st.primary_rays, st.shadow_rays, st.reflection_rays))
    shape = refs[0].shape
    fb = int(np.prod(shape)) * 4
    bufs = [torch.empty((4,) + shape, dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    pa = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC, **kw)
    rays = lambda s: (s.primary_rays, s.shadow_rays, s.reflection_rays)  # noqa: E731
    # (batch cameras) per step: equal, then mixed, then moved, then 3-frame batches
    plan = [[0, 0, 0, 0]] * 3 + [[0, 1, 2, 3]] * 2 + [[3, 2, 1, 0]] + [[1, 1, 2]] * 2
    try:
        for k, sel in enumerate(plan):
            for lone in (False, True):
                n = 2 if not lone else 1  # two batches in flight, then one at a time
                for i in range(n):
                    ctx.set_stream(streams[i].cuda_stream)
                    ctx.render_device_batch([cams[j] for j in sel], fr.plane, pa, bufs[i].data_ptr(), fb)
                launch = ctx.last_launch()
                st = ctx.finish()
                torch.cuda.synchronize()
                assert launch.startswith("render_batch_kernel<"), launch
                assert f"frames={len(sel)}" in launch, launch
                for i in range(n):
                    got = bufs[i].cpu().numpy()
                    for f, j in enumerate(sel):
                        assert np.array_equal(got[f].view(np.uint32), refs[j].view(np.uint32)), (k, lone, i, f, launch)
                want = tuple(n * sum(rst[j][q] for j in sel) for q in range(3))
                assert rays(st) == want, (k, lone, launch)
    finally:
        ctx.set_stream(None)
        ctx.close()


def test_batch_falls_back_to_single_frames(gpu_ctx, rt):
    """Frames a batch launch does not cover (here 1 spp and 16 spp) are
    rendered one by one by rt_render_device_batch: same bits and counts."""
    import torch
    for spp in (1, 16):
        fr = rt.make("C3").with_resolution(160, 90).with_(spp=spp)
        gpu_ctx.set_scene(fr.scene)
        ref, sr = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
        fb = ref.size * 4
        buf = torch.empty((3,) + ref.shape, dtype=torch.float32, device="cuda")
        st = gpu_ctx.render_device_batch([fr.camera] * 3, fr.plane, rt.frame_params(fr), buf.data_ptr(), fb)
        got = buf.cpu().numpy()
        for f in range(3):
            assert np.array_equal(got[f].view(np.uint32), ref.view(np.uint32)), (spp, f)
        assert (st.primary_rays, st.shadow_rays) == (3 * sr.primary_rays, 3 * sr.shadow_rays), spp
        assert not gpu_ctx.last_launch().startswith("render_batch_kernel"), gpu_ctx.last_launch()


@pytest.mark.parametrize("band", [(1, 4), (0, 2), (5, 8)])
def test_shares_in_flight_equal_row_major(gpu_ctx, rt, band):
    """One rank's share of a C3 frame, frames in flight on two streams (the
    bench's --sim-bands case): shares of more than 24,000 tiles (1/2, 1/4)
    take the 6-wave split instance and sky batches, a 1/8 share the 5-wave
    one — every frame equals the row-major share frame bit for bit."""
    import torch
    fr = rt.make("C3")
    # a context of its own: a context keeps longest-first state for 16
    # (stream, slab) pairs, and the shared one has met many streams by now
    ctx = rt.Context()
    ctx.set_scene(fr.scene)
    bi, bn = band
    kw = dict(band_index=bi, band_count=bn, band_rows=8)
    row, sr = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
    outs = [torch.empty(row.shape, dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    pa = rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC, **kw)
    try:
        launches = []
        for f in range(12):
            k = f % 2
            ctx.set_stream(streams[k].cuda_stream)
            ctx.render_device(fr.camera, fr.plane, pa, outs[k].data_ptr(), outs[k].numel() * 4)
            launches.append(ctx.last_launch())
            if k == 1:
                st = ctx.finish()
                torch.cuda.synchronize()
                for i in range(2):
                    assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), row.view(np.uint32)), (f, i)
                assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == tuple(
                    2 * v for v in (sr.primary_rays, sr.shadow_rays, sr.reflection_rays)), f
        tiles = int(launches[-1].split("tiles=")[1].split()[0])
        w = 6 if tiles > 24000 else 5
        assert launches[-1].startswith(f"render_kernel<false, true, false, true, {w}, false>"), launches[-1]
        assert (int(launches[-1].split("sky=")[1].split()[0]) > 0) == (tiles > 24000), launches[-1]
    finally:
        ctx.set_stream(None)
        ctx.close()


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C5"])
@pytest.mark.parametrize("cap", [0, 40, 1])
def test_one_sample_waves_trace_with_the_whole_wave(gpu_ctx, rt, name, cap):
    """A lone shard's slowest pixels run as one-sample waves whose whole wave
    traces the sample's ray chain (trace.hip render_sample_wave, coop.h: 16
    stack entries tested per step, four lanes each): same bits and ray counts
    as row-major frames, on the mesh / sphere / loose-triangle scenes (C5 at 4
    spp, the megakernel's), with wide steps up to the whole stack area (cap
    0), up to 40 entries (a mix of wide and depth-first steps) and never (1:
    every step depth-first, one entry)."""
    fr = rt.make(name)
    if fr.spp != 4:
        fr = fr.with_(spp=4)
    fr = fr.with_resolution(480, 270)
    gpu_ctx.set_scene(fr.scene)
    lib = gpu_ctx.lib
    assert lib.rt_debug_set(gpu_ctx.h, rt.abi.RT_DEBUG_SAMPLE_WAVE_STACK, cap) == 0
    try:
        for kw in ({}, dict(band_index=2, band_count=3, band_rows=8)):
            row, sr = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
            for _ in range(3):  # the first frame measures and sorts; later ones split
                img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, **kw))
                assert np.array_equal(img.view(np.uint32), row.view(np.uint32)), kw
                assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (sr.primary_rays, sr.shadow_rays,
                                                                                 sr.reflection_rays), kw
            assert "s16_shift=0" in gpu_ctx.last_launch(), gpu_ctx.last_launch()
    finally:
        assert lib.rt_debug_set(gpu_ctx.h, rt.abi.RT_DEBUG_SAMPLE_WAVE_STACK, 0) == 0


def test_one_sample_handoff_under_concurrent_streams(rt):
    """The one-sample waves' relaxed hand-off (trace.hip split_handoff: the
    samples by agent-scope stores, a wait, a relaxed count, the last arrival's
    agent-scope loads) with other work on the GPU: four contexts, each on its
    own stream, render lone 1/8 shares of C3 concurrently (each frame is lone
    in its context, so it runs one-sample waves: s16_shift=0), frame after
    frame; every pixel of every frame equals the unsplit row-major share.  Band 7
    is the ragged one (135 row blocks: its 17th lies past the image), so the rows
    inside the image are compared: a share's padding rows are not part of the
    image (rt_band_rows_local)."""
    import torch
    from unity_raytracer_amd.bands import band_global_rows
    fr = rt.make("C3")
    ctxs, streams, outs, refs, keep = [], [], [], [], []
    try:
        for k in range(4):
            c = rt.Context()
            c.set_scene(fr.scene)
            kw = dict(band_index=2 * k + 1, band_count=8, band_rows=8)
            ref, _ = c.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
            s = torch.cuda.Stream()
            c.set_stream(s.cuda_stream)
            ctxs.append((c, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC, **kw)))
            streams.append(s)
            outs.append(torch.empty(ref.shape, dtype=torch.float32, device="cuda"))
            keep.append(band_global_rows(fr.plane.ResolutionY, 2 * k + 1, 8, 8) >= 0)
            assert keep[-1].shape == (ref.shape[0],)
            refs.append(ref[keep[-1]])
        assert not keep[3].all()  # the ragged band's padding block
        for f in range(8):
            for k, (c, p) in enumerate(ctxs):
                outs[k].fill_(float("nan"))
            torch.cuda.synchronize()
            for k, (c, p) in enumerate(ctxs):  # enqueued back to back: the four run at once
                c.render_device(fr.camera, fr.plane, p, outs[k].data_ptr(), outs[k].numel() * 4)
            for k, (c, p) in enumerate(ctxs):
                c.finish()
            torch.cuda.synchronize()
            for k, (c, p) in enumerate(ctxs):
                if f >= 2:  # from the third frame on the order exists and the slowest pixels run as one-sample waves
                    assert "s16_shift=0" in c.last_launch(), c.last_launch()
                got = outs[k].cpu().numpy()[keep[k]]
                assert np.array_equal(got.view(np.uint32), refs[k].view(np.uint32)), (f, k)
    finally:
        for c, _ in ctxs:
            c.set_stream(None)
            c.close()


def test_split_sixteenths_of_large_shards_is_invisible(gpu_ctx, rt):
    """Shards of 24,000-70,000 tiles (a 1/2 and a 1/4 shard of 1080p C3) run
    their slowest tiles finely split — synchronous (lone) frames their slowest
    1/1024, the 1/4 shard (<= 40,000 tiles) as one-sample waves, the 1/2 shard
    as one-pixel waves — and a whole synchronous 1080p frame its slowest
    1/4096 as one-pixel waves (the 6-wave split instance): same bits and ray
    counts as row-major frames."""
    fr = rt.make("C3")
    gpu_ctx.set_scene(fr.scene)
    for kw in (dict(band_index=0, band_count=2, band_rows=8), dict(band_index=3, band_count=4, band_rows=8), {}):
        row, sr = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
        for _ in range(3):
            img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, **kw))
            assert np.array_equal(img.view(np.uint32), row.view(np.uint32)), kw
            assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == (sr.primary_rays, sr.shadow_rays,
                                                                             sr.reflection_rays), kw
