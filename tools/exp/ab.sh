# A/B of library variants: probe timings on configs, then the TCC write/read
# request pass per variant on C3 (HBM bytes per launch of the Q4 megakernel).
# usage: bash tools/exp/ab.sh <tag> <variants> <configs>
set -o pipefail
tag=$1; vars=$2; cfgs=$3
R=$GRAFT_REPO_ROOT
bash $R/tools/exp/probe.sh $tag $vars $cfgs || exit 1
cd /tmp && export TMPDIR=/tmp
for v in ${vars//,/ }; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ --output-format csv \
    -d $R/gpurun_out/pmcw_${tag}_$v -o run -- python3 $R/tools/probe.py --config C3 --modes megakernel --frames 3 --variants $v \
    > $R/gpurun_out/pmcw_${tag}_$v.log 2>&1 || { echo pmc-fail-$v; exit 1; }
  python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcw_${tag}_$v --kernel "render_kernel<false, false, false, true>" \
    --out $R/gpurun_out/pmcw_${tag}_$v.json > /dev/null && python3 -c "
import json; d=json.load(open('$R/gpurun_out/pmcw_${tag}_$v.json')); c=d['counters']
print('$v', 'wr_req', c.get('TCC_EA0_WRREQ'), 'wr64', c.get('TCC_EA0_WRREQ_64B'), 'rd_req', c.get('TCC_EA0_RDREQ'))"
done
echo AB-DONE
