# Round-4 GPU session 6: the adopted changes (lean setup, split-instance
# occluder hints, levels-kernel LDS stash, split synchronous frames) — GPU
# suite, interleaved A/B against the session's base build, bench line, kernel
# trace and the C3 / C4 counter passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 300 python tools/abx.py --config C3 --variants base,default,st8w6,leaf4 --rounds 10 --frames 12 \
  > gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants base,default --rounds 10 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b8-fail; exit 1; }
for c in C4 C5 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants base,default,lvhi9,xcd,leaf4 --rounds 6 --frames 6 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$tag -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 > $R/gpurun_out/kt_$tag.log 2>&1 || { echo kt-fail; exit 1; }
cd $R
for cb in C3:1 C4:1; do
  bash tools/pmc_round.sh $tag ${cb%%:*} ${cb##*:} > gpurun_out/pmcr_${tag}_${cb%%:*}.log 2>&1 || { echo pmc-fail-$cb; tail gpurun_out/pmcr_${tag}_${cb%%:*}.log; exit 1; }
done
echo ALLDONE
