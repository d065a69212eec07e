# Round-4 GPU session 18: LDS pixel sums in the levels kernel (C4, C5); then
# a diagnostic of the one-sample split-wave build (s64rt) on the multi-device
# group tests, which stalled in r04s (verbose, short per-test timeout).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04t}
for c in C5 C4; do
  timeout -k 10 400 python tools/abx.py --config $c --variants default,ldssum --rounds 4 --frames 3 \
    >> gpurun_out/abx_lds_$tag.log 2>&1 || { echo abx-lds-fail; tail gpurun_out/abx_lds_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_lds_$tag.log
RT_TEST_LIB_VARIANT=s64rt timeout -k 10 240 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 60 --timeout-method thread \
  > gpurun_out/tests_s64rt_$tag.log 2>&1 || { echo s64rt-tests-fail; tail -60 gpurun_out/tests_s64rt_$tag.log; exit 1; }
tail -3 gpurun_out/tests_s64rt_$tag.log
echo ALLDONE
