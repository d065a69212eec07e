# Round-4 GPU session 17: one-sample split waves in the product (shards):
# GPU suite, A/B against r04o (the round's previous final) and without the
# lone-shard rule (s64nolone), wave clocks.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04s}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants r04o,default,s64nolone --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants r04o,default --rounds 6 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 > gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-fail; tail gpurun_out/wclk_$tag.log; exit 1; }
for c in C5 C4; do
  timeout -k 10 400 python tools/abx.py --config $c --variants default,ldssum --rounds 4 --frames 3 \
    >> gpurun_out/abx_lds_$tag.log 2>&1 || { echo abx-lds-fail; tail gpurun_out/abx_lds_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_lds_$tag.log
echo ALLDONE
