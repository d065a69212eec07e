cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in default; do
  timeout -k 10 100 python tools/e2e_probe.py --config C3 --frames 20 --variant $v >> gpurun_out/e2e2.log 2>&1 || { echo fail $v; tail -5 gpurun_out/e2e2.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/e2e2.log
