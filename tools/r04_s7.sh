# Round-4 GPU session 7: megakernel occupancy (per-lane LDS stack vs waves per
# SIMD), the synchronous-frame split, and the XCD-aware levels dispatch.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04h}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,st8w6,st16w6,st8w7,w6ns,ns --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default,st8w6,st16w6,st8w7 --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b8-fail; exit 1; }
for c in C4 C5; do
  timeout -k 10 300 python tools/abx.py --config $c --variants base,default --rounds 5 --frames 6 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
