cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="timeout -k 10 120 python tools/probe.py --config C3 --modes megakernel,rowmajor --frames 20"
$P --variants default,seg > gpurun_out/p1.log 2>&1 &&
$P --variants default,seg --bounces 0 >> gpurun_out/p1.log 2>&1 &&
$P --variants default,seg --no-lights >> gpurun_out/p1.log 2>&1 &&
$P --variants default,seg --no-lights --bounces 0 >> gpurun_out/p1.log 2>&1
cat gpurun_out/p1.log | grep -v amdgpu.ids
