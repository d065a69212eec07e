set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { echo bench-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof-fail; exit 1; }
P="python3 tools/probe.py --config C3 --modes megakernel --frames 3"
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B -d gpurun_out/pmcA -o p --output-format csv -- $P > gpurun_out/pmcA.log 2>&1 || { echo pmcA-fail; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_HIT TCC_MISS -d gpurun_out/pmcB -o p --output-format csv -- $P > gpurun_out/pmcB.log 2>&1 || { echo pmcB-fail; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmcC -o p --output-format csv -- $P > gpurun_out/pmcC.log 2>&1 || { echo pmcC-fail; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM -d gpurun_out/pmcD -o p --output-format csv -- $P > gpurun_out/pmcD.log 2>&1 || { echo pmcD-fail; exit 1; }
echo all-ok
