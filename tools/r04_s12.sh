# Round-4 GPU session 12: final-build measurements.
#   a: GPU suite, smoke, bench line, kernel traces (default bench command and
#      --streams 1), wave clocks, levels segments, e2e probe with mapped output
#   b: counter passes (C3 whole / 1/2 / 1/4 / 1/8, C4, C5 whole and 1/8)
#   c: one-rank shares, C4/C5 bench lines, round A/B against the round's base
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04m}
stage=${2:-a}
if [ "$stage" = a ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { echo smoke-fail; tail gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || { echo bench-fail; tail -20 gpurun_out/bench_$tag.log; exit 1; }
echo bench-ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$tag -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/kt_$tag.log 2>&1 || { echo kt-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kts1_$tag -o run --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 > $R/gpurun_out/kts1_$tag.log 2>&1 || { echo kts1-fail; exit 1; }
echo kt-ok
cd $R
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 > gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-fail; tail gpurun_out/wclk_$tag.log; exit 1; }
for c in C4 C5; do
  timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 --variants seglv,default \
    >> gpurun_out/seglv_$tag.log 2>&1 || { echo seglv-$c-fail; tail gpurun_out/seglv_$tag.log; exit 1; }
done
for fl in 8 0; do
  timeout -k 10 200 python tools/e2e_probe.py --config C3 --frames 12 --flags $fl --mapped >> gpurun_out/e2e_$tag.log 2>&1 || { echo e2e-fail; tail gpurun_out/e2e_$tag.log; exit 1; }
done
echo stage-a-ok
fi
if [ "$stage" = b ]; then
for cb in C3:1 C3:2 C3:4 C3:8 C4:1 C4:8 C5:1 C5:8; do
  bash tools/pmc_round.sh $tag ${cb%%:*} ${cb##*:} > gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log 2>&1 || { echo pmc-fail-$cb; tail gpurun_out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log; exit 1; }
  echo pmc-ok-$cb
done
fi
if [ "$stage" = c ]; then
for c in C4 C5; do
  timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 --variants seglv \
    >> gpurun_out/seglv_${tag}c.log 2>&1 || { echo seglv-$c-fail; tail gpurun_out/seglv_${tag}c.log; exit 1; }
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_$tag.log 2>&1 || { echo sb$n-fail; exit 1; }
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands $n --streams 1 > gpurun_out/sb${n}s1_$tag.log 2>&1 || { echo sb${n}s1-fail; exit 1; }
done
echo sb-ok
for c in C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 > gpurun_out/bench_${c}_$tag.log 2>&1 || { echo bench-$c-fail; exit 1; }
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 --sim-bands 8 > gpurun_out/sb8_${c}_$tag.log 2>&1 || { echo sb8-$c-fail; exit 1; }
done
echo cfg-ok
for c in C3 C2 C4 C5; do
  timeout -k 10 300 python tools/abx.py --config $c --variants base,default --rounds 6 --frames 8 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants base,default --rounds 6 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b-fail; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
fi
echo ALLDONE
