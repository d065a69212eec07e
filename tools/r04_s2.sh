# Round-4 GPU session 2: what the sky tiles cost with frames in flight
# (waves dropped / sky stores skipped), lean setup on a 1/8 band.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04b}
timeout -k 10 300 python tools/abx.py --config C3 --variants default,lean,droptail,skynostore,skypass,skypass_lean --rounds 8 --frames 12 \
  > gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default,lean,lastocc --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b8-fail; exit 1; }
grep variant gpurun_out/abx_$tag.log

RT_TEST_LIB_VARIANT=skypass_lean timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cut.py \
  tests/test_gpu_sky.py tests/test_gpu_host_out.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_skypass_$tag.log 2>&1 || { echo tests-skypass-fail; tail -30 gpurun_out/tests_skypass_$tag.log; exit 1; }
tail -1 gpurun_out/tests_skypass_$tag.log
echo ALLDONE
