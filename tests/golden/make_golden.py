"""Generate tests/golden/frames.npz — committed golden frames for the demo
scene (RayTracing.unity, 50x50) and config C1 (256x256).

The reference (C#/Unity) cannot run here, so the frames come from the C
oracle (oracle/rt_oracle.c) and are accepted only if the independent numpy
restatement (oracle/np_oracle.py) reproduces them BIT FOR BIT; the per-
function known answers that pin the oracle itself are hand-derived in
tests/golden/kat.json (incl. the reference's own t = 299 case,
Assets/RayTracer/Tests/RayTracerTests.cs:11-26).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import _rt_pkg  # noqa: E402

rt = _rt_pkg.load()
orc = _rt_pkg.load_oracle()
import np_oracle  # noqa: E402


def main():
    out = {}
    for name in ("demo", "C1"):
        fr = rt.make(name)
        a, ca = orc.render(fr)
        b, cb = np_oracle.render(fr)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), name
        assert all(ca[k] == cb[k] for k in cb), name
        out[name] = a[..., :3].copy()
        out[name + "_counts"] = np.array([ca["primary_rays"], ca["shadow_rays"], ca["reflection_rays"]], np.int64)
        print(name, a.shape, ca)
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **out)


if __name__ == "__main__":
    main()
