"""The conservative sky test at the Scene.AABB silhouette.

A wave whose every sample, approximated with fast reciprocals, misses the
Scene.AABB padded by 2^-10 of the camera-relative scene scale is answered as
background without its exact rays (shade.h sky_maybe, rt_frame.cpp
sky_setup).  The reference's exact gate is RMath.RayAABBIntersection on
Scene.AABB (RMath.cs:12-26, Scene.cs:54): a wrong decision would turn a whole
tile of pixels into background.  Here hundreds of seeded cameras per scene
aim at random points of the box's edges and corners with narrow fields of view
and odd resolutions, so the silhouette crosses tiles at sub-pixel offsets
(and partial edge tiles), for the general render_kernel (1 spp), its 2x2-spp
instance (4 spp) and the <= 16-spp level-synchronous kernel (16 spp).  Every
frame must be bit-identical to the counting launch of the same frame (which
never sky-tests) and, on the silhouette pixels, to the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CAMERAS = 200


def scene_box(sc):
    pts = [m.AABB.reshape(-1, 3).astype(np.float64) for m in sc.Meshes]
    if len(sc.TriangleData.Triangles):
        pts.append(np.asarray(sc.TriangleData.Triangles, np.float64).reshape(-1, 3))
    sp = np.asarray(sc.SphereData.Spheres, np.float64).reshape(-1, 4)
    if len(sp):
        r = np.sqrt(sp[:, 3:4])
        pts += [sp[:, :3] - r, sp[:, :3] + r]
    p = np.concatenate(pts)
    return p.min(0), p.max(0)


def sample_dirs(fr):
    """Every sample ray direction of the frame (float64, unnormalised), (H, W, spp, 3)."""
    cam, pl = fr.camera, fr.plane
    W, H, n = pl.ResolutionX, pl.ResolutionY, int(round(np.sqrt(fr.spp)))
    pos, fwd = np.asarray(cam.Position, np.float64), np.asarray(cam.Forward, np.float64)
    right, up = np.asarray(cam.Right, np.float64), np.asarray(cam.Up, np.float64)
    tl = (pos + fwd * pl.DistanceToCamera - right * pl.HalfHorizontalLength) + up * pl.HalfVerticalLength
    ys, xs = np.mgrid[0:H, 0:W]
    out = np.empty((H, W, n * n, 3))
    for sj in range(n):
        for si in range(n):
            rx = (xs + (si + 0.5) / n) * 2 * pl.HalfHorizontalLength / W
            ry = (ys + (sj + 0.5) / n) * 2 * pl.HalfVerticalLength / H
            out[:, :, sj * n + si] = tl + rx[..., None] * right - ry[..., None] * up - pos
    return out


def hits_box(pos, d, lo, hi):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1, t2 = (lo - pos) * inv, (hi - pos) * inv
        tmin = np.maximum(np.nanmax(np.minimum(t1, t2), -1), 0.0)
        tmax = np.nanmin(np.maximum(t1, t2), -1)
    return tmin <= tmax


def silhouette_frames(rt, base, seed, n, lo, hi):
    """n frames whose Scene.AABB silhouette crosses the image: cameras outside
    the box aimed at a random point of a random box edge, random roll, narrow
    random field of view, odd resolutions, 1 / 4 / 16 spp in turn."""
    rng = np.random.default_rng(seed)
    S = rt.scenes
    diag = float(np.linalg.norm(hi - lo))
    frames = []
    tries = 0
    while len(frames) < n and tries < 50 * n:
        tries += 1
        a = int(rng.integers(3))
        tgt = np.where(rng.integers(0, 2, 3) == 1, hi, lo).astype(np.float64)
        tgt[a] = rng.uniform(lo[a], hi[a])
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        pos = tgt + d * diag * rng.uniform(0.7, 4.0)
        if np.all(pos >= lo - 0.05 * diag) and np.all(pos <= hi + 0.05 * diag):
            continue  # the sky test is off with the camera inside the padded box
        fwd = tgt - pos + rng.normal(size=3) * diag * 1e-3
        fwd /= np.linalg.norm(fwd)
        up0 = rng.normal(size=3)
        right = np.cross(up0, fwd)
        if np.linalg.norm(right) < 1e-3:
            continue
        right /= np.linalg.norm(right)
        up = np.cross(fwd, right)
        spp = (1, 4, 16)[len(frames) % 3]
        rx, ry = int(rng.integers(9, 41)), int(rng.integers(7, 33))
        hh = float(rng.uniform(0.03, 0.5))
        f32 = lambda v: tuple(float(x) for x in np.asarray(v, np.float32))  # noqa: E731
        fr = base.with_(camera=S.CameraData(Position=f32(pos), Forward=f32(fwd), Right=f32(right), Up=f32(up)),
                        plane=S.ImagePlane(ResolutionX=rx, ResolutionY=ry, DistanceToCamera=1.0,
                                           HalfHorizontalLength=hh, HalfVerticalLength=hh * ry / rx),
                        spp=spp)
        hit = hits_box(np.asarray(fr.camera.Position, np.float64), sample_dirs(fr), lo, hi)
        if hit.any() and not hit.all():
            frames.append((fr, hit))
    assert len(frames) == n, f"only {len(frames)} silhouette cameras in {tries} tries"
    return frames


def silhouette_pixels(hit):
    """Pixels whose samples, or whose 8 neighbours' samples, disagree on the box."""
    px = hit.any(-1).astype(np.int8) + hit.all(-1).astype(np.int8)  # 0 miss, 1 mixed, 2 all hit
    H, W = px.shape
    pad = np.pad(px, 1, mode="edge")
    mn = np.min([pad[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)], axis=0)
    mx = np.max([pad[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)], axis=0)
    return np.flatnonzero((mn != mx).ravel())


def translated(rt, fr, off):
    import copy

    o = np.asarray(off, np.float32)
    sc = copy.deepcopy(fr.scene)
    td = sc.TriangleData
    if len(td.Triangles):
        td.Triangles = (td.Triangles + o).astype(np.float32)
    for m in sc.Meshes:
        m.Triangles = (m.Triangles + o).astype(np.float32)
        m.AABB = (m.AABB + o).astype(np.float32)
    if len(sc.SphereData.Spheres):
        sc.SphereData.Spheres[:, :3] = (sc.SphereData.Spheres[:, :3] + o).astype(np.float32)
    if len(sc.PointLights):
        sc.PointLights[:, :3] = (sc.PointLights[:, :3] + o).astype(np.float32)
    return fr.with_(scene=sc)


@pytest.mark.parametrize("name,seed", [("C2", 101), ("C3", 202), ("C5", 303), ("far", 404)])
def test_sky_test_at_the_silhouette(rt, gpu_ctx, orc, name, seed):
    if name == "far":  # a small scene far from the origin: large camera-relative coordinates
        base = translated(rt, rt.make("C1"), (900.0, -350.0, 1200.0))
    else:
        base = rt.make(name)
    base = base.with_(max_bounces=min(base.max_bounces, 4))
    gpu_ctx.set_scene(base.scene)
    lo, hi = scene_box(base.scene)
    b4 = None
    if name in ("C3", "C5"):  # the oracle walks the exported tree (equal to the brute-force scan)
        nodes, tris, sphs = gpu_ctx.export_bvh()
        b4 = orc.Bvh4Scene(base, nodes, tris, sphs)
    checked = 0
    try:
        for k, (fr, hit) in enumerate(silhouette_frames(rt, base, seed, CAMERAS, lo, hi)):
            img, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
            ref, _ = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS))
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), \
                f"{name} camera {k} spp {fr.spp}: sky-tested frame != counting launch (no sky test)"
            idx = silhouette_pixels(hit)
            if k % 4 == 0 and len(idx):  # the oracle on a quarter of the cameras' silhouettes
                if b4 is not None:
                    b4.fr = fr
                    want, _ = b4.render_pixels(idx.astype(np.int32))
                else:
                    want, _ = orc.render_pixels(fr, idx.astype(np.int32))
                got = img.reshape(-1, 4)[idx]
                assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
                    f"{name} camera {k}: silhouette pixels != oracle"
                checked += len(idx)
    finally:
        if b4 is not None:
            b4.close()
    assert checked > 0
