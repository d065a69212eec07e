# Round-3 GPU session 1: tests, bench, segment clocks, kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/tests_s1.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_s1.log; exit 1; }
tail -3 gpurun_out/tests_s1.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s1.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_s1.log; exit 1; }
tail -1 gpurun_out/bench_s1.log | cut -c1-600
timeout -k 10 300 python tools/probe.py --config C3 --modes megakernel --variants default,seg --frames 10 > gpurun_out/seg_s1.log 2>&1 || { echo seg-fail; exit 1; }
cat gpurun_out/seg_s1.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_s1 -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 > $R/gpurun_out/kt_s1.log 2>&1 || { echo kt-fail; exit 1; }
echo ALLDONE
