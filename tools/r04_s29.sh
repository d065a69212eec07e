# Round-4 GPU session 29: final library (one-sample split waves for lone
# shards only) — round-end rehearsal (smoke, bench with no flags), one rank's
# shares with frames in flight and one at a time, A/B against round 3's base.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ak}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke-fail; tail gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rehearsal_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_rehearsal_$tag.log; exit 1; }
grep '^{' gpurun_out/bench_rehearsal_$tag.log | cut -c1-200
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_$tag.log 2>&1 || { echo sb$n-fail; exit 1; }
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands $n --streams 1 > gpurun_out/sb${n}s1_$tag.log 2>&1 || { echo sb${n}s1-fail; exit 1; }
done
echo sb-ok
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants base,default --rounds 6 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
