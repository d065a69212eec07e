# usage: bash tools/exp/pmc.sh <tag> <variant> <config> [probe args]   (SQ passes only)
set -o pipefail
tag=$1; var=$2; cfg=$3; shift 3
EXTRA=("$@")
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_$tag
run() {
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $R/gpurun_out/pmc_$tag/$1 -o run -- \
    python3 $R/tools/probe.py --config $cfg --modes megakernel --frames 3 --variants $var "${EXTRA[@]}" > $R/gpurun_out/pmc_$tag/$1.log 2>&1
}
run C "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" &&
run D "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM" &&
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_$tag/C $R/gpurun_out/pmc_$tag/D --kernel "render_kernel<false, false>" --out $R/gpurun_out/pmc_$tag/summary.json > /dev/null &&
python3 -c "
import json; d=json.load(open('$R/gpurun_out/pmc_$tag/summary.json'))
c=d.get('counters',{}); print('$tag', {k: round(v/1e6,2) for k,v in sorted(c.items())})"
