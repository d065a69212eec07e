"""bench.py end to end on the GPU (subprocesses, as the driver runs it): the
single-GPU line's schema, and the distributed frame loop — grouped RCCL
gathers of row shards, partial groups, one reassembly launch per group —
at one rank over RCCL and at two ranks over gloo, each checked with
`--verify` (the reassembled frame must equal a single-rank frame bit for
bit)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, timeout=150, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    return p


def _metric_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def _verified(stderr):
    return any(json.loads(l).get("verify_sharded_equals_single") is True
               for l in stderr.splitlines() if l.startswith('{"verify'))


def test_bench_single_gpu_line():
    p = _run([sys.executable, "bench.py", "--steps", "4", "--warmup", "1", "--no-cpu-baseline"])
    d = _metric_line(p.stdout)
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1 and d["unit"] == "Mrays/s"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"]
    c = d["config"]
    assert c["resolution"] == "1920x1080" and c["spp"] == 4 and c["depth"] == 8
    assert c["rays_per_frame"] > 1920 * 1080 * 4  # primary + shadow + mirror rays
    assert c["end_to_end_ms_per_frame"] > c["kernel_ms_per_frame"] > 0


def test_bench_rccl_path_one_rank_partial_groups():
    # 7 timed frames in groups of 4 (one partial group); 3 warmup frames
    p = _run([sys.executable, "bench.py", "--steps", "7", "--warmup", "3", "--no-cpu-baseline", "--force-dist",
              "--verify", "--gather-frames", "4"], env_extra={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())})
    assert _verified(p.stderr), p.stderr[-3000:]
    d = _metric_line(p.stdout)
    assert d["config"]["frames_per_gather"] == 4 and "RCCL" in d["config"]["parallelism"]


def test_bench_gloo_two_ranks_one_gpu():
    p = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
              "--steps", "5", "--warmup", "1", "--dist-backend", "gloo", "--verify", "--no-cpu-baseline",
              "--gather-frames", "2"], timeout=240)
    assert _verified(p.stderr), p.stderr[-3000:]
    d = _metric_line(p.stdout)
    assert d["n_gpus"] == 2 and d["config"]["frames_per_gather"] == 2


def test_bench_spawns_gloo_ranks_without_launcher():
    """`bench.py --gpus 2` with no launcher starts its own two ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--dist-backend", "gloo", "--verify", "--no-cpu-baseline", "--gather-frames", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert _verified(p.stderr), p.stderr[-3000:]
    assert _metric_line(p.stdout)["n_gpus"] == 2


def test_bench_in_process_multi_device():
    """One process, one multi-device context (logical shards on GPU 0): the
    library's own band gather, verified against a one-device frame."""
    p = _run([sys.executable, "bench.py", "--in-process", "--devices", "0,0,0", "--steps", "4", "--warmup", "1",
              "--verify"], timeout=240)
    assert _verified(p.stderr), p.stderr[-3000:]
    d = _metric_line(p.stdout)
    assert "peer-copy" in d["config"]["parallelism"] and d["value"] > 0
