# kernel trace of the per-Update rebuild loop (C3)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/rbtr -o run -- \
  python3 $R/tools/exp/rebuild_one.py > $R/gpurun_out/rbtr.log 2>&1
