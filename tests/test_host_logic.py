"""Host-side logic that needs no GPU: the longest-first cost key of split
tiles (rt_device.h tile_cost_key, compiled for the host with hipcc) and
bench.py's own rank launcher."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _key(c):
    """Python restatement of the unsplit key (log scale, 4 mantissa bits)."""
    c = min(c, 0xFFFFFFFF)
    e = c.bit_length() - 1 if c else 0
    return c if e < 4 else (((e - 3) << 4) | ((c >> (e - 4)) & 15))


def test_split_tile_cost_key(tmp_path):
    """A tile split into 64 >> pshift parts is charged its first part's cost
    times the number of parts (it was charged 4x too much)."""
    prog = tmp_path / "k.hip"
    prog.write_text(r'''
#include <cstdio>
#include "rt_device.h"
int main() {
    const unsigned long long cs[] = {0, 1, 7, 15, 16, 17, 1000, 123456, 4000000000ull, 1ull << 40};
    for (unsigned long long c : cs)
        for (int ps : {2, 4})
            std::printf("%llu %d %u %u %u\n", c, ps, rtd::tile_cost_key(c, -1, ps), rtd::tile_cost_key(c, 0, ps),
                        rtd::tile_cost_key(c, 1, ps));
    return 0;
}''')
    exe = tmp_path / "k"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-host-only", "-std=c++17", "-I",
                    os.path.join(ROOT, "unity-raytracer_amd", "csrc"), "-o", str(exe), str(prog)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    n = 0
    for line in filter(None, out):
        c, ps, whole, first, other = map(int, line.split())
        parts = 64 >> ps
        assert whole == _key(c)
        assert first == _key(c * parts), (c, ps)  # first part x parts
        assert other == _key(c)  # only part 0 is recorded by the kernel; the key itself is unscaled
        n += 1
    assert n == 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_spawns_its_own_ranks():
    """`bench.py --gpus 2` without a launcher starts two ranks itself
    (torch.distributed.run, before any GPU call) and they form one group."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    seen = sorted((d["rank"], d["world"]) for d in
                  (json.loads(l) for l in p.stderr.splitlines() if l.startswith('{"launch_check"')))
    assert seen == [(0, 2), (1, 2)], p.stderr[-3000:]


def test_bench_rejects_world_size_mismatch():
    """A launcher whose world size differs from --gpus is an error, not a
    silently single-GPU number."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--launch-check"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE 2" in p.stderr


def test_bench_canonical_check_without_counts():
    """profiles/canonical_counts.json pins only fetched bytes for C4 (no
    oracle walk of a 4K frame): bench.py --config C4 reports the canonical
    counts as missing instead of failing (r07s)."""
    sys.path.insert(0, ROOT)
    import bench

    class St:
        primary_rays = shadow_rays = reflection_rays = box_tests = triangle_tests = sphere_tests = 0
        shading_fetches = 0

    entries = json.load(open(os.path.join(ROOT, "profiles", "canonical_counts.json")))
    assert "C4" in entries and "counts" not in entries["C4"]
    assert bench.canonical_check("C4", St(), True) == {"state": "missing"}
    assert bench.canonical_check("C3", St(), True)["state"] == "mismatch"
    assert bench.canonical_check("C3", St(), False)["state"] == "n/a (row band)"
