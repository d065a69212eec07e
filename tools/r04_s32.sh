# Round-4 GPU session 32: issue priority 3 for the one-sample waves of
# <= 24,000-tile shards (the product build) against the previous library;
# GPU suite and counter passes at the new library.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04an}
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants prev,default --rounds 10 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
bash tools/r04_s12.sh $tag b
