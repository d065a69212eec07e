# Round-4 GPU session 23: the device LBVH's leaf rule (node-step cost against
# a primitive test: 0.5 / 1 (default) / 2 / 3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04aa}
for c in C5 C3 C4 C2; do
  timeout -k 10 400 python tools/abx.py --config $c --variants default,lc05,lc20,lc30 --rounds 4 --frames 6 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
