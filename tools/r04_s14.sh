# Round-4 GPU session 14: readlane sample sums (levels kernel epilogue) against r04o.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sky.py tests/test_gpu_counts.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
for c in C5 C4; do
timeout -k 10 500 python tools/abx.py --config $c --variants r04o,default --rounds 4 --frames 3 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
for c in C4 C5; do
  timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 --variants seglv \
    >> gpurun_out/seglv_$tag.log 2>&1 || { echo seglv-$c-fail; tail gpurun_out/seglv_$tag.log; exit 1; }
done
echo ALLDONE
