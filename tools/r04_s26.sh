# Round-4 GPU session 26: tile rows per XCD stripe of the levels kernel's
# dispatch (1 / 2 / 4 (default) / 8 / 16) on C5 and C4.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ad}
for c in C5 C4; do
  timeout -k 10 500 python tools/abx.py --config $c --variants default,xr1,xr2,xr8,xr16 --rounds 4 --frames 4 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
