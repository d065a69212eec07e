# Round-4 GPU session 38: how many of a <= 24,000-tile shard's slowest tiles
# run as sixteenth (lone: one-sample) waves — 1/2048 (default), 1/1024, 1/4096.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04av}
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default,sd1024,sd4096 --rounds 10 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
