# usage: bash tools/exp/r03_ab.sh <tag> <variants> <configs> [tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
tag=$1; vars=$2; cfgs=$3
bash tools/exp/probe.sh $tag $vars $cfgs || exit 1
if [ "${4:-}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -2 gpurun_out/tests_$tag.log
fi
echo AB-DONE
