"""The oracle's traversal of a 4-wide tree in the GPU's record layout
(rt_device.h: 128-B nodes, 48-B triangle / 32-B sphere records; the CPU leg
"bvh_same_tree" of bench.py) on CPU: a small hand-built tree over the demo
scene and C1 must render exactly the brute-force frames (Scene.IntersectRay,
Data/Objects/Scene.cs:43-122).  The GPU test tests/test_gpu_bvh_export.py
does the same with the trees the library builds."""
import struct

import numpy as np

PAD = 1e-3


def _leaf_ref(first, count, kind):
    return ~(first | ((count - 1) << 27) | (kind << 29))


def _node(children):
    """children: list of (lo3, hi3, ref) (<= 4); empty slots +inf boxes -> sentinel leaf."""
    lo = np.full((3, 4), np.inf, np.float32)
    hi = np.full((3, 4), -np.inf, np.float32)
    refs = [0, 0, 0, 0]
    for i, (l, h, r) in enumerate(children):
        lo[:, i] = np.asarray(l, np.float32) - PAD
        hi[:, i] = np.asarray(h, np.float32) + PAD
        refs[i] = r
    b = b""
    for a in range(3):
        b += lo[a].tobytes() + hi[a].tobytes()
    b += struct.pack("<4i", *refs) + struct.pack("<4i", 0, 0, 0, 0)
    assert len(b) == 128
    return b


def _build(scene):
    """Root over one leaf child per <= 4 primitives (homogeneous in kind and
    mesh), in a two-level tree when there are more than 4 leaves."""
    tri_recs, sph_recs, leaves = [], [], []
    MT = sum(len(m.Triangles) for m in scene.Meshes)
    NS = len(scene.SphereData.Spheres)

    def tri_rec(t, rank, gate):
        v0, v1, v2 = t.astype(np.float32)
        e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
        f = np.array([v0[0], v0[1], v0[2], e1[0], e1[1], e1[2], e2[0], e2[1], e2[2]], np.float32)
        return f[:9].tobytes() + struct.pack("<2i", rank, gate) + b"\0" * 4

    rank = 0
    for mi, m in enumerate(scene.Meshes):
        tris = np.asarray(m.Triangles, np.float32)
        for s in range(0, len(tris), 4):
            chunk = tris[s:s + 4]
            first = len(tri_recs)
            for k, t in enumerate(chunk):
                tri_recs.append(tri_rec(t, rank + s + k, mi))
            pts = chunk.reshape(-1, 3)
            leaves.append((pts.min(0), pts.max(0), _leaf_ref(first, len(chunk), 0)))
        rank += len(tris)
    for i, sp in enumerate(np.asarray(scene.SphereData.Spheres, np.float32)):
        r = float(np.sqrt(sp[3]))
        sph_recs.append(sp.tobytes() + struct.pack("<4i", MT + i, -1, 0, 0))
        leaves.append((sp[:3] - r, sp[:3] + r, _leaf_ref(len(sph_recs) - 1, 1, 1)))
    loose = np.asarray(scene.TriangleData.Triangles, np.float32)
    for s in range(0, len(loose), 4):
        chunk = loose[s:s + 4]
        first = len(tri_recs)
        for k, t in enumerate(chunk):
            tri_recs.append(tri_rec(t, MT + NS + s + k, -1))
        pts = chunk.reshape(-1, 3)
        leaves.append((pts.min(0), pts.max(0), _leaf_ref(first, len(chunk), 0)))
    sentinel = len(tri_recs)
    tri_recs.append(b"\0" * 36 + struct.pack("<2i", 0x7fffffff, -1) + b"\0" * 4)  # zero edges: never hit
    # pad empty slots with the sentinel leaf
    groups = [leaves[i:i + 4] for i in range(0, len(leaves), 4)]
    nodes = []
    if len(groups) == 1:
        nodes.append(_node(groups[0]))
    else:
        assert len(groups) <= 4
        kids = []
        for gi, g in enumerate(groups):
            lo = np.min([c[0] for c in g], 0)
            hi = np.max([c[1] for c in g], 0)
            kids.append((lo, hi, 1 + gi))
        nodes.append(_node(kids))
        nodes += [_node(g) for g in groups]
    fixed = []
    for nb in nodes:  # unused slots point at the sentinel triangle (as the library does)
        refs = list(struct.unpack("<4i", nb[96:112]))
        lo0 = np.frombuffer(nb[0:16], np.float32)
        for i in range(4):
            if not np.isfinite(lo0[i]):
                refs[i] = _leaf_ref(sentinel, 1, 0)
        fixed.append(nb[:96] + struct.pack("<4i", *refs) + nb[112:])
    as_u8 = lambda bs: np.frombuffer(b"".join(bs), np.uint8) if bs else np.zeros(0, np.uint8)  # noqa: E731
    assert all(len(r) == 48 for r in tri_recs) and all(len(r) == 32 for r in sph_recs)
    return as_u8(fixed), as_u8(tri_recs), as_u8(sph_recs)


def test_bvh4_oracle_equals_brute_force(rt, orc):
    for name, res in (("demo", None), ("C1", (64, 48))):
        fr = rt.make(name)
        if res:
            fr = fr.with_resolution(*res)
        nodes, tris, sphs = _build(fr.scene)
        b4 = orc.Bvh4Scene(fr, nodes, tris, sphs)
        try:
            idx = np.arange(fr.plane.ResolutionX * fr.plane.ResolutionY, dtype=np.int32)
            got, cg = b4.render_pixels(idx, threads=2)
            ref, cr = orc.render_pixels(fr, idx, threads=2)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), name
            for k in ("primary_rays", "shadow_rays", "reflection_rays"):
                assert cg[k] == cr[k], (name, k)
        finally:
            b4.close()
