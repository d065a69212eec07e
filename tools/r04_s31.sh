# Round-4 GPU session 31: issue priority for one-sample split waves (lone
# 1/8 and 1/4 shares, one frame at a time).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04am}
for b in 0/8 0/4; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,prio1,prio3 --rounds 10 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
