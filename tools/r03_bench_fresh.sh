# Bench lines of the final library with its hash-gated PMC summaries in place
# (profiles/pmc_*.json): C3 default line, C4 / C5 whole frames, C4 / C5 one-rank
# 1/8 shares, the RCCL path at one rank.  usage: bash tools/r03_bench_fresh.sh <tag>
set -o pipefail
tag=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bf_${tag}_C3.log 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 > gpurun_out/bf_${tag}_C4.log 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 > gpurun_out/bf_${tag}_C5.log 2>&1 &&
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline --sim-bands 8 > gpurun_out/bf_${tag}_sb8C4.log 2>&1 &&
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline --sim-bands 8 > gpurun_out/bf_${tag}_sb8C5.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --force-dist --verify > gpurun_out/bf_${tag}_fd.log 2>&1 &&
echo ALLDONE
