# Round-4 GPU session 21: host SAH against the device LBVH tree for the
# levels-kernel configs (C5: 20,833 scattered meshes; C4) and C3/C2.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04w}
for c in C5 C4 C3 C2; do
  timeout -k 10 400 python tools/abx.py --config $c --variants default,default@lbvh --rounds 4 --frames 4 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
