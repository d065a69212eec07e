# Round-4 GPU session 16: do one-sample waves shorten a shard's slowest chain?
# one0..one3: timing-only variants (each traces one sample of a split pixel,
# wrong images); s64: split tiles as 64 one-sample waves whose pixel sums meet
# through write-through stores and an arrival count (bit-identical).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04r}
RT_TEST_LIB_VARIANT=s64 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py tests/test_gpu_cut.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_s64_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_s64_$tag.log; exit 1; }
tail -1 gpurun_out/tests_s64_$tag.log
for b in 0/8 0/4; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,s64,one0,one1,one2,one3 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,s64 --rounds 6 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
