# rocprofv3 runtime + kernel + memory-copy trace of synchronous rt_render frames
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for cfg in "0 8" "8 3"; do set -- $cfg
timeout -k 10 200 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/e2etr_$1_$2 -o run -- \
  python3 $R/tools/exp/e2e_one.py $1 $2 10 > $R/gpurun_out/e2etr_$1_$2.log 2>&1 || { echo fail-$1; exit 1; }
done
echo done
