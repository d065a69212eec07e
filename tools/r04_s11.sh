# Round-4 GPU session 11: levels-kernel camera packets from the top-level cut
# (lvcut: 64-spp instance, lvcut2: both) and 8 waves/SIMD for 64 spp (lv8).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04l}
RT_TEST_LIB_VARIANT=lvcut2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cut.py tests/test_gpu_sky.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_lvcut2_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_lvcut2_$tag.log; exit 1; }
tail -1 gpurun_out/tests_lvcut2_$tag.log
timeout -k 10 500 python tools/abx.py --config C5 --variants default,lvcut,lvcut2,lv8 --rounds 4 --frames 3 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-C5-fail; tail gpurun_out/abx_$tag.log; exit 1; }
timeout -k 10 500 python tools/abx.py --config C4 --variants default,lvcut2 --rounds 4 --frames 3 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-C4-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
