# One PMC pass: VALU/SALU issue and wave-state counters of the C3 megakernel.
# usage (GPU box): bash tools/pmc_valu.sh <tag> [probe args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcv_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcv_$tag -o run -- \
  python $R/tools/probe.py --config C3 --modes megakernel --frames 3 "$@" > $R/gpurun_out/pmcv_$tag/probe.log 2>&1
