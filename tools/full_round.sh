# Whole-state GPU session (on the box): tests, bench, gloo rehearsals, other
# configs (tools/gpu_round.sh), a single-stream rocprofv3 kernel trace, the
# PMC passes, one rank's share at N = 2/4/8, and the RCCL path at one rank.
# usage: bash tools/full_round.sh <tag>
set -o pipefail
tag=${1:-cur}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$tag -o run -- \
  python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 > $R/gpurun_out/kt_$tag.log 2>&1 || { echo kt-fail; exit 1; }
cd $R
bash tools/pmc_round.sh $tag || { echo pmc-fail; exit 1; }
cd $R
for n in 2 4 8; do
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_$tag.log 2>&1 || { echo sb$n-fail; exit 1; }
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --force-dist --verify > gpurun_out/fd_$tag.log 2>&1 || { echo fd-fail; exit 1; }
echo ALLDONE
