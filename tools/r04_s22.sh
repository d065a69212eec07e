# Round-4 GPU session 22: the device LBVH as rt_set_scene's default — GPU
# suite, canonical counts of the new trees (C2, C3, C5; oracle walk ==
# counting launch), A/B against r04o (host SAH default).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04x}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 600 python -u tools/canonical_counts.py --configs C2,C3,C5 --out gpurun_out/canonical_counts.json \
  > gpurun_out/canonical_$tag.log 2>&1 || { echo canonical-fail; tail gpurun_out/canonical_$tag.log; exit 1; }
echo canonical-ok
for c in C3 C5 C4 C2; do
  timeout -k 10 400 python tools/abx.py --config $c --variants r04o,default --rounds 4 --frames 6 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
