# Round-4 GPU session 3: the whole GPU suite (incl. the canonical-count and
# sky-silhouette tests), the canonical per-config counts at full size, and the
# sky-tile cost A/B (frames in flight).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
timeout -k 10 400 python tools/canonical_counts.py --configs C2,C3,C5 --out gpurun_out/canonical_counts.json \
  > gpurun_out/canonical_$tag.log 2>&1 || { echo canonical-fail; tail -5 gpurun_out/canonical_$tag.log; exit 1; }
grep -c '"equal": true' gpurun_out/canonical_$tag.log
bash tools/r04_s2.sh $tag
