# Round-4 GPU session 13: the 64-spp levels instance — LDS stash of the
# shadow-packet state (9 / 15 floats) at 8 and 7 waves/SIMD; time and writes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04n}
timeout -k 10 600 python tools/abx.py --config C5 --variants default,w7,hi9,hi15,hi15w7 --rounds 4 --frames 3 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-C5-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
for v in hi15 hi15w7; do
  VARIANT=$v bash tools/pmc_round.sh $tag C5 1 > gpurun_out/pmcr_${tag}_C5_$v.log 2>&1 || { echo pmc-fail-$v; tail gpurun_out/pmcr_${tag}_C5_$v.log; exit 1; }
  echo pmc-ok-$v
done
timeout -k 10 300 python tools/exp/e2e_variants.py --flags 8 --variants default,sw_1,sw_3_1,sw_6_1,sw_2_2_1,sw_4_2_1_1 > gpurun_out/e2e_sw_$tag.log 2>&1 || { echo e2e8-fail; tail gpurun_out/e2e_sw_$tag.log; exit 1; }
timeout -k 10 300 python tools/exp/e2e_variants.py --flags 0 --variants default,sw_1,sw_1_1_2_2_3_3,sw_1_2_3_4,sw_1_1_2_3_9 >> gpurun_out/e2e_sw_$tag.log 2>&1 || { echo e2e0-fail; tail gpurun_out/e2e_sw_$tag.log; exit 1; }
grep -v amdgpu gpurun_out/e2e_sw_$tag.log
for b in 0/2 0/4; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,lone1024,lone2048 --rounds 8 --frames 12 \
    >> gpurun_out/abx_lone_$tag.log 2>&1 || { echo abx-lone-fail; exit 1; }
done
grep variant gpurun_out/abx_lone_$tag.log
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 > gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-fail; tail gpurun_out/wclk_$tag.log; exit 1; }
echo ALLDONE
