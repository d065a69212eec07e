# Round-4 GPU session 35: the split fraction of lone whole frames (and of
# 1/2 shares with frames in flight): 1/2048, 1/4096 (default), 1/8192.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04aq}
timeout -k 10 300 python tools/abx.py --config C3 --variants default,lg2048,lg8192 --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/2 --variants default,lg2048,lg8192 --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
