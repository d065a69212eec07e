# Round-4 GPU session 37: the split fraction of lone whole frames, fewer still —
# 1/16384 (default), 1/32768, one tile (1/131072) — and C2 beside it.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04au}
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,wh32768,wh131072 --rounds 10 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
