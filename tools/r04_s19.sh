# Round-4 GPU session 19: the whole GPU suite on the one-sample split-wave
# build (s64rt), verbose, to find the test that stalled in r04s.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04u}
RT_TEST_LIB_VARIANT=s64rt timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread \
  > gpurun_out/tests_s64rt_$tag.log 2>&1 || { echo s64rt-suite-fail; tail -80 gpurun_out/tests_s64rt_$tag.log; exit 1; }
tail -3 gpurun_out/tests_s64rt_$tag.log
echo ALLDONE
