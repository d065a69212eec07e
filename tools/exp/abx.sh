# usage: bash tools/exp/abx.sh <tag> <variants> <configs> [tests] — interleaved A/B (tools/abx.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
tag=$1; vars=$2; cfgs=$3
for c in ${cfgs//,/ }; do
  timeout -k 10 300 python tools/abx.py --config $c --variants $vars >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail-$c; tail -5 gpurun_out/abx_$tag.log; exit 1; }
done
grep '"variant"' gpurun_out/abx_$tag.log
if [ "${4:-}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -2 gpurun_out/tests_$tag.log
fi
echo AB-DONE
