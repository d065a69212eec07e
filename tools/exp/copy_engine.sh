# rt_render (row slabs + D2H copies) under the HIP runtime's copy-engine flags:
# default, blit workgroups limited, SDMA forced for every size, blit engine types.
# usage: bash tools/exp/copy_engine.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-ce}
cd $R
run() {
  echo "== $1" >> gpurun_out/ce_$tag.log
  env $2 timeout -k 10 120 python tools/e2e_probe.py --config C3 --frames 12 >> gpurun_out/ce_$tag.log 2>&1 || { echo fail-$1; return 1; }
}
run default "RT_DUMMY=0" &&
run limwg16 "DEBUG_CLR_LIMIT_BLIT_WG=16" &&
run limwg64 "DEBUG_CLR_LIMIT_BLIT_WG=64" &&
run forcesdma "GPU_FORCE_BLIT_COPY_SIZE=0" &&
run engine1 "GPU_BLIT_ENGINE_TYPE=1" &&
run engine2 "GPU_BLIT_ENGINE_TYPE=2" || exit 1
grep -v amdgpu.ids gpurun_out/ce_$tag.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/ce_${tag}_trace -o run -- \
  python3 $R/tools/e2e_probe.py --config C3 --frames 6 > $R/gpurun_out/ce_${tag}_trace.log 2>&1 || echo trace-fail
echo CE-DONE
