# Interleaved A/B (tools/abx.py) of library variants on the given configs.
# usage: bash tools/exp/ab_cfg.sh <tag> <variants> <configs comma-separated> [tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
tag=$1; vars=$2; cfgs=$3
mkdir -p gpurun_out
if [ "${4:-}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -1 gpurun_out/tests_$tag.log
fi
for c in ${cfgs//,/ }; do
  fr=10; [ $c = C4 ] || [ $c = C5 ] && fr=4
  timeout -k 10 300 python tools/abx.py --config $c --variants $vars --rounds 8 --frames $fr \
    > gpurun_out/ab_${tag}_$c.jsonl 2>&1 || { echo ab-fail-$c; tail -5 gpurun_out/ab_${tag}_$c.jsonl; exit 1; }
  grep variant gpurun_out/ab_${tag}_$c.jsonl | cut -c1-300
done
echo ALLDONE
