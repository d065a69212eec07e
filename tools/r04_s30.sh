# Round-4 GPU session 30: how many of a lone 1/4 (and 1/2) share's slowest
# tiles to split (one-sample waves at <= 40,000 tiles): 1/1024 .. 1/128.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04al}
for b in 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,l512,l256,l128 --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
echo ALLDONE
