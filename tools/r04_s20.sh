# Round-4 GPU session 20: round-end rehearsal on the final build (GPU suite,
# smoke, the default bench line with its counter roofline), then the GPU suite
# again on the one-sample split-wave build (s64rt) for stability evidence.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04v}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke-fail; tail gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
grep '^{' gpurun_out/bench_$tag.log | cut -c1-400
RT_TEST_LIB_VARIANT=s64rt timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread \
  > gpurun_out/tests_s64rt_$tag.log 2>&1 || { echo s64rt-suite-fail; tail -80 gpurun_out/tests_s64rt_$tag.log; exit 1; }
tail -1 gpurun_out/tests_s64rt_$tag.log
echo ALLDONE
