# On the GPU box: the demo frame through the host-ASan/UBSan build of the whole
# library (tools/asan/Makefile `gpu`, built beforehand on the CPU), compared
# bit for bit with the committed golden frame.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  timeout -k 10 120 tools/asan/build/cast_pixel_rays gpurun_out/asan_demo.f32 > gpurun_out/asan_gpu.log 2>&1 || { echo asan-run-fail; tail -40 gpurun_out/asan_gpu.log; exit 1; }
python3 - <<'PY' >> gpurun_out/asan_gpu.log
import numpy as np
img = np.fromfile("gpurun_out/asan_demo.f32", np.float32).reshape(50, 50, 4)
g = np.load("tests/golden/frames.npz")["demo"]
print("demo frame == golden:", bool(np.array_equal(img[..., :3].view(np.uint32), g.view(np.uint32))))
PY
cat gpurun_out/asan_gpu.log
