# Camera-packet cut start: GPU tests, interleaved A/B against the HEAD build
# (lib/variants/base) on C3 / C4 / C5, segment clocks of the new build.
# usage: bash tools/exp/cut_ab.sh <tag> [notests]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
tag=${1:-cut}
mkdir -p gpurun_out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -1 gpurun_out/tests_$tag.log
fi
for c in C3 C2 C4 C5; do
  fr=10; [ $c = C4 ] || [ $c = C5 ] && fr=4
  timeout -k 10 300 python tools/abx.py --config $c --variants base,default --rounds 8 --frames $fr \
    > gpurun_out/ab_${tag}_$c.jsonl 2>&1 || { echo ab-fail-$c; tail -5 gpurun_out/ab_${tag}_$c.jsonl; exit 1; }
  cat gpurun_out/ab_${tag}_$c.jsonl | cut -c1-400
done
timeout -k 10 300 python tools/probe.py --config C3 --modes megakernel --variants seg --frames 10 > gpurun_out/seg_$tag.log 2>&1 || { echo seg-fail; exit 1; }
cat gpurun_out/seg_$tag.log
echo ALLDONE
