# Round-4 GPU session 4: the levels kernel (C4 / C5) with the shadow-packet
# lane state in LDS (lvstash) against the default build: interleaved A/B and
# the HBM write counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04d}
for c in C4 C5; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,lvstash,lvstash6 --rounds 6 --frames 6 \
    >> gpurun_out/abx_lv_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_lv_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_lv_$tag.log
for v in default lvstash; do
  VARIANT=$v bash tools/pmc_round.sh $tag C4 1 > gpurun_out/pmcr_${tag}_C4_$v.log 2>&1 || { echo pmc-$v-fail; tail gpurun_out/pmcr_${tag}_C4_$v.log; exit 1; }
done

for c in C3 C5 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,sah2,sah4 --rounds 6 --frames 8 \
    >> gpurun_out/abx_sah_$tag.log 2>&1 || { echo abx-sah-$c-fail; tail gpurun_out/abx_sah_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_sah_$tag.log
echo S4DONE
