# Round-3 GPU session 2 (on the box): per-segment cycle split of a C3 wave at
# HEAD (segment-clock build through tools/probe.py), then the one-rank PMC
# passes, sim-bands shares, C4/C5 benches and the RCCL path (tools/r03_full.sh
# without its tests, bench and kernel trace steps).
# usage: bash tools/r03_s2.sh <tag>
set -o pipefail
tag=${1:-cur}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe.py --config C3 --modes megakernel --variants default,seg --frames 10 > gpurun_out/seg_$tag.log 2>&1 || { echo seg-fail; tail gpurun_out/seg_$tag.log; exit 1; }
tail -2 gpurun_out/seg_$tag.log | cut -c1-700
for cb in C3:8 C4:8 C5:8; do
  bash tools/pmc_round.sh $tag ${cb%%:*} ${cb##*:} > gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log 2>&1 || { echo pmc-fail-$cb; tail gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log; exit 1; }
  echo pmc-ok-$cb
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_$tag.log 2>&1 || { echo sb$n-fail; exit 1; }
done
for c in C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --sim-bands 8 > gpurun_out/sb8_${c}_$tag.log 2>&1 || { echo sb8-$c-fail; exit 1; }
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 > gpurun_out/bench_${c}_$tag.log 2>&1 || { echo bench-$c-fail; exit 1; }
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --force-dist --verify > gpurun_out/fd_$tag.log 2>&1 || { echo fd-fail; exit 1; }
echo ALLDONE
