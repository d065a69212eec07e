# usage: bash tools/exp/sdma.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-sd}
cd $R
timeout -k 10 120 python tools/exp/sdma_probe.py --config C3 > gpurun_out/sdma_$tag.log 2>&1 || { echo probe-fail; tail gpurun_out/sdma_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sdma_$tag.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/sdma_${tag}_trace -o run -- \
  python3 $R/tools/exp/sdma_probe.py --config C3 --reps 2 > $R/gpurun_out/sdma_${tag}_trace.log 2>&1 || echo trace-fail
echo SD-DONE
