# Round-3 whole-state GPU session (on the box): GPU tests, smoke, bench line,
# a single-stream rocprofv3 kernel trace of the bench, the PMC passes of the
# trace kernel for C3 / C4 / C5 (whole frame and one rank's 1/8 band), the
# one-rank shares at N = 2/4/8 (C3) and N = 8 (C4, C5), and the RCCL path at
# one rank.  Every step has its own time limit; the first failure ends it.
# usage: [PMCS="C3:1 C4:1"] [SIMS=0] bash tools/r03_full.sh <tag> [notests]
set -o pipefail
tag=${1:-cur}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -1 gpurun_out/tests_$tag.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke-fail; tail gpurun_out/smoke_$tag.log; exit 1; }
  tail -1 gpurun_out/smoke_$tag.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
echo bench-ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$tag -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 > $R/gpurun_out/kt_$tag.log 2>&1 || { echo kt-fail; exit 1; }
echo kt-ok
cd $R
for cb in ${PMCS:-C3:1 C3:8 C4:1 C4:8 C5:1 C5:8}; do
  bash tools/pmc_round.sh $tag ${cb%%:*} ${cb##*:} > gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log 2>&1 || { echo pmc-fail-$cb; tail gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log; exit 1; }
  echo pmc-ok-$cb
done
[ "${SIMS:-1}" = 0 ] && { echo ALLDONE; exit 0; }
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_$tag.log 2>&1 || { echo sb$n-fail; exit 1; }
done
for c in C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --sim-bands 8 > gpurun_out/sb8_${c}_$tag.log 2>&1 || { echo sb8-$c-fail; exit 1; }
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 > gpurun_out/bench_${c}_$tag.log 2>&1 || { echo bench-$c-fail; exit 1; }
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --force-dist --verify > gpurun_out/fd_$tag.log 2>&1 || { echo fd-fail; exit 1; }
echo ALLDONE
