# PMC passes for the default C3 megakernel (one counter group per rocprofv3
# run, --kernel-trace only alongside; MI355X_MICROARCH.md "rocprofv3 PMC slots").
# usage (on the GPU box): bash tools/pmc_round.sh <tag>
set -o pipefail
tag=${1:-cur}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  # one counter group per rocprofv3 run
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $R/gpurun_out/pmc_$tag/$1 -o run -- \
    python3 $R/tools/probe.py --config C3 --modes megakernel --frames 3 > $R/gpurun_out/pmc_$tag/$1.log 2>&1
}
mkdir -p $R/gpurun_out/pmc_$tag
run A "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ" &&
run B "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_HIT TCC_MISS" &&
run C "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" &&
run D "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM" &&
python $R/tools/pmc_summary.py $R/gpurun_out/pmc_$tag/A $R/gpurun_out/pmc_$tag/B $R/gpurun_out/pmc_$tag/C $R/gpurun_out/pmc_$tag/D \
  --kernel "render_kernel<false, false, false, true>" --out $R/gpurun_out/pmc_$tag/summary.json > /dev/null && echo pmc-ok
