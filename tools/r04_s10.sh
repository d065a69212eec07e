# Round-4 GPU session 10: mirror chains of split waves as packets (pchain:
# every split instance, pchain5: the shard instance only) — parity of the
# variant on the split/cut/parity tests, A/B against the default, wave clocks.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04k}
RT_TEST_LIB_VARIANT=pchain timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cut.py tests/test_gpu_bench.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_pchain_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_pchain_$tag.log; exit 1; }
tail -1 gpurun_out/tests_pchain_$tag.log
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,pchain,pchain5 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,pchain,pchain5 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b-fail; exit 1; }
done
timeout -k 10 300 python tools/abx.py --config C2 --band 0/8 --variants default,pchain,pchain5 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-c2b-fail; exit 1; }
grep variant gpurun_out/abx_$tag.log
for v in wclk wclk_pc; do
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,8 --variant $v >> gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-fail; tail gpurun_out/wclk_$tag.log; exit 1; }
done
echo ALLDONE
