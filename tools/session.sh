# One GPU-box session (run on the box from the repo root):
#   bash tools/session.sh <tag> [tests|notests]
# GPU tests, the default bench line, a single-stream rocprofv3 kernel trace of
# the bench, and the PMC passes of the C3 trace kernel (tools/pmc_round.sh),
# each step under its own time limit; the first failure ends the session.
set -o pipefail
tag=${1:-cur}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  echo tests-ok
fi
if [ -x tools/asan/build/cast_pixel_rays ]; then bash tools/asan/run_gpu.sh > gpurun_out/asan_$tag.txt 2>&1 || { echo asan-fail; tail gpurun_out/asan_$tag.txt; exit 1; }; fi
echo asan-ok
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
echo bench-ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$tag -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 > $R/gpurun_out/kt_$tag.log 2>&1 || { echo kt-fail; exit 1; }
echo kt-ok
cd $R
bash tools/pmc_round.sh $tag || { echo pmc-fail; exit 1; }
echo ALLDONE
