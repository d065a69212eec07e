# Round-4 GPU session 24: whole-frame megakernel occupancy re-measured on the
# device-LBVH tree (5 / 6 (default) / 7 waves per SIMD).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ab}
for c in C3 C2; do
  timeout -k 10 400 python tools/abx.py --config $c --variants default,mw5,mw7 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
