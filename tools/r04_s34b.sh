# Round-4 GPU session 34: round-end rehearsal at the committed final library
# and counter files (smoke, bench with no flags, the GPU suite once more).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ap}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke-fail; tail gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rehearsal_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_rehearsal_$tag.log; exit 1; }
grep '^{' gpurun_out/bench_rehearsal_$tag.log | cut -c1-200
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
echo ALLDONE
