# Round-4 GPU session 2: what the sky tiles cost with frames in flight
# (waves dropped / sky stores skipped), lean setup on a 1/8 band.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04b}
timeout -k 10 300 python tools/abx.py --config C3 --variants default,lean,droptail,skynostore --rounds 8 --frames 12 \
  > gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default,lean,lastocc --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b8-fail; exit 1; }
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
