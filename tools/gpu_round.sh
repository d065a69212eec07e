# One GPU-box session: parity tests, bench, kernel trace, multi-rank rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo bench-fail; exit 1; }
for n in 2 3; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 1 --dist-backend gloo --verify > gpurun_out/bench_gloo$n.log 2>&1 || { echo gloo$n-fail; exit 1; }
done
for c in C2 C4 C5; do timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 >> gpurun_out/probe_cfg.log 2>&1 || { echo probe-$c-fail; exit 1; }; done
echo all-ok
