# rt_render into host memory: its GPU tests, the e2e probe (C3 float and
# RGBA8), then the whole GPU suite.  usage: bash tools/exp/host_out.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-st}
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_host_out.py > gpurun_out/host_tests_$tag.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/host_tests_$tag.log; exit 1; }
tail -3 gpurun_out/host_tests_$tag.log
for fl in 0 8; do
timeout -k 10 120 python tools/e2e_probe.py --config C3 --frames 12 --flags $fl >> gpurun_out/host_e2e_$tag.log 2>&1 || { echo e2e-fail; exit 1; }
done
grep -v amdgpu.ids gpurun_out/host_e2e_$tag.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/host_all_$tag.log 2>&1 || { echo all-fail; tail -30 gpurun_out/host_all_$tag.log; exit 1; }
tail -2 gpurun_out/host_all_$tag.log
echo HO-DONE
