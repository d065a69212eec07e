# Round-4 GPU session 1: GPU tests on the current build, interleaved A/B of the
# C3 megakernel variants (lean setup, last-occluder hints), segment clocks,
# and the 1/8-share critical path (slowest wave) for synchronous frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04a}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 400 python tools/abx.py --config C3 --variants r03,default,lean,lastocc,both --rounds 8 --frames 10 \
  > gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
timeout -k 10 200 python tools/probe.py --config C3 --modes megakernel --frames 10 --variants seg,seg_both \
  > gpurun_out/seg_$tag.log 2>&1 || { echo seg-fail; exit 1; }
timeout -k 10 200 python tools/probe.py --config C3 --modes megakernel --frames 10 --variants segmax \
  > gpurun_out/segmax_$tag.log 2>&1 || { echo segmax-fail; exit 1; }
for b in 2 4 8; do
  timeout -k 10 200 python tools/probe.py --config C3 --modes megakernel --frames 10 --variants segmax --band 0/$b \
    >> gpurun_out/segmax_$tag.log 2>&1 || { echo segmax-b$b-fail; exit 1; }
done
timeout -k 10 300 python tools/abx.py --config C3 --variants default,split16all --rounds 6 --frames 10 \
  > gpurun_out/abx_split_$tag.log 2>&1 || { echo abx-split-fail; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default,both --rounds 6 --frames 10 \
  >> gpurun_out/abx_split_$tag.log 2>&1 || { echo abx-b8-fail; exit 1; }
grep variant gpurun_out/abx_split_$tag.log
echo ALLDONE
