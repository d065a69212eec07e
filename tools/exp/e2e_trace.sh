cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/e2etr -o run -- python3 $R/tools/e2e_probe.py --config C3 --frames 6 > $R/gpurun_out/e2etr.log 2>&1 || { echo fail; tail $R/gpurun_out/e2etr.log; exit 1; }
ls -R $R/gpurun_out/e2etr | head
