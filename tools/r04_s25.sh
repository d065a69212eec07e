# Round-4 GPU session 25: the 64-spp levels instance's camera packets from the
# top-level cut, now on the device-LBVH tree (its Morton-ordered top levels
# overlap less than the SAH tree's, where the cut measured C5 +43 %).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ac}
timeout -k 10 400 python tools/abx.py --config C5 --variants default,lvcuthi --rounds 4 --frames 4 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
