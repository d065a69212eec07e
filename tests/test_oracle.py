"""The CPU oracle pinned against hand-derived known answers, the committed
golden frames and an independent numpy restatement (CPU only)."""
import json
import math
import os
import struct

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))


@pytest.mark.parametrize("case", KAT["sphere"], ids=lambda c: c["name"])
def test_kat_sphere(orc, case):
    hit, t = orc.ray_sphere(case["ray"], case["sphere"])
    assert hit == case["hit"]
    if hit:
        assert t == np.float32(case["t"])


@pytest.mark.parametrize("case", KAT["triangle"], ids=lambda c: c["name"])
def test_kat_triangle(orc, case):
    hit, t = orc.ray_triangle(case["ray"], case["tri"])
    assert hit == case["hit"]
    if hit:
        assert t == np.float32(case["t"])


@pytest.mark.parametrize("case", KAT["aabb"], ids=lambda c: c["name"])
def test_kat_aabb(orc, case):
    assert orc.ray_aabb(case["ray"], case["box"]) == case["hit"]


@pytest.mark.parametrize("case", KAT["triangle_normal"], ids=lambda c: c["name"])
def test_kat_triangle_normal(orc, rt, case):
    n = orc.triangle_normal(case["tri"])
    assert np.array_equal(n, np.array(case["normal"], np.float32))
    # the host-side extraction helper (product) agrees
    m = rt.scene.triangle_normal(np.array(case["tri"], np.float32).reshape(1, 3, 3))[0]
    assert np.array_equal(m, n)


def test_golden_frames(orc, rt):
    g = np.load(os.path.join(HERE, "golden", "frames.npz"))
    for name in ("demo", "C1"):
        img, counts = orc.render(rt.make(name))
        assert np.array_equal(img[..., :3].view(np.uint32), g[name].view(np.uint32)), name
        assert (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]) == tuple(g[name + "_counts"])
        assert np.all(img[..., 3] == 1.0)


@pytest.mark.parametrize("name,res,spp", [("demo", None, 4), ("C2", (48, 27), 4), ("C1", (40, 30), 9)])
def test_numpy_restatement_bit_exact(orc, rt, name, res, spp):
    import np_oracle
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=spp)
    a, ca = orc.render(fr)
    b, cb = np_oracle.render(fr)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for k in cb:
        assert ca[k] == cb[k]


def test_render_pixels_matches_frame(orc, rt):
    fr = rt.make("C2").with_resolution(64, 36)
    full, _ = orc.render(fr)
    idx = np.array([0, 5, 64 * 10 + 7, 64 * 36 - 1], np.int32)
    px, _ = orc.render_pixels(fr, idx)
    assert np.array_equal(px, full.reshape(-1, 4)[idx])
    rows, _ = orc.render_rows(fr, 3, 5)
    assert np.array_equal(rows, full[3::5])


def _f(bits):
    return struct.unpack("<f", struct.pack("<I", bits))[0]


def _key(f):
    b = struct.unpack("<I", struct.pack("<f", f))[0]
    return -(b & 0x7FFFFFFF) if b & 0x80000000 else b


def _from_key(k):
    return _f((0x80000000 | -k) if k < 0 else k)


def _backfacing_py(d):
    return np.float32(math.acos(d)) * np.float32(57.29578) > np.float32(90)


def test_spec_threshold(orc, rt):
    """degrees(acos(d)) > 90f (RayTracingSetup.cs:384-392) == d < T for the
    library's T (rt_spec_threshold, host function — no GPU needed), checked
    exhaustively over every float within 2^20 ulps of T and on a coarse
    sweep of [-1, 1]."""
    lib = rt.load_library()
    lib.rt_spec_threshold.restype = __import__("ctypes").c_float
    T = lib.rt_spec_threshold()
    kT = _key(T)
    ks = np.arange(kT - (1 << 20), kT + (1 << 20), dtype=np.int64)
    bits = np.where(ks < 0, 0x80000000 | (-ks), ks).astype(np.uint32)
    d = bits.view(np.float32)
    back = np.float32(np.arccos(d.astype(np.float64))).astype(np.float32) * np.float32(57.29578) > np.float32(90)
    assert np.array_equal(back, d < np.float32(T))
    for x in np.linspace(-1, 1, 2001, dtype=np.float32):
        assert orc.spec_backfacing(float(x)) == bool(x < np.float32(T))
    for x in (-1.0, -0.5, -1e-7, -0.0, 0.0, 1e-7, 0.5, 1.0):
        assert orc.spec_backfacing(x) == bool(np.float32(x) < np.float32(T))


def test_encode_rgba8_known_answers():
    import np_oracle as npo
    c = np.array([[0.5, 0.0, 1.0, 1.0], [-1.0, 2.0, np.nan, 1.0], [np.inf, -np.inf, 0.25, 1.0],
                  [1.5 / 255, 2.5 / 255, 0.2 / 255, 1.0]], np.float32)
    got = npo.encode_rgba8(c)
    want = np.array([[128, 0, 255, 255], [0, 255, 0, 255], [255, 0, 64, 255], [2, 2, 0, 255]], np.uint8)
    # 0.5*255 = 127.5 -> 128 (even); 0.25*255 = 63.75 -> 64; 1.5/255*255 rounds to 1.5 -> 2 (even),
    # 2.5/255*255 -> 2.5 -> 2 (even)
    assert np.float32(np.float32(1.5 / 255) * np.float32(255)) == np.float32(1.5)
    assert np.float32(np.float32(2.5 / 255) * np.float32(255)) == np.float32(2.5)
    assert np.array_equal(got, want)
    h = npo.encode_rgba16f(c[:1])
    assert h.dtype == np.float16 and h[0, 0] == np.float16(0.5) and h[0, 3] == 1


@pytest.mark.parametrize("name,res", [("demo", None), ("C1", (64, 48)), ("C2", (64, 36)), ("C3", (48, 27)),
                                      ("C5", (32, 18))])
def test_cpu_bvh_mode_equals_brute_force(orc, rt, name, res):
    """The CPU-baseline BVH mode (oracle/rt_oracle.c orc_bvh_*) answers like the scan."""
    fr = rt.make(name)
    if res:
        fr = fr.with_resolution(*res)
    fr = fr.with_(spp=1, max_bounces=min(fr.max_bounces, 3))
    idx = np.arange(fr.plane.ResolutionX * fr.plane.ResolutionY, dtype=np.int32)
    ref, rc = orc.render_pixels(fr, idx)
    b = orc.BvhScene(fr)
    got, gc = b.render_pixels(idx)
    b.close()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert (gc["primary_rays"], gc["shadow_rays"], gc["reflection_rays"]) == \
        (rc["primary_rays"], rc["shadow_rays"], rc["reflection_rays"])


def test_cpu_bvh_mode_fuzz(orc, rt):
    import test_gpu_fuzz
    for seed in range(12):
        fr = test_gpu_fuzz.random_frame(rt, seed, res=(20, 15), spp=1, bounces=seed % 4)
        idx = np.arange(300, dtype=np.int32)
        ref, _ = orc.render_pixels(fr, idx)
        b = orc.BvhScene(fr)
        got, _ = b.render_pixels(idx)
        b.close()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), seed
