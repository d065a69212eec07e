# Round-4 GPU session 9: split-instance changes (whole-frame split without
# occluder hints, moot shadow rays in split chains, 24-entry stacks at five
# waves, lone-stream async frames split) against the r04i build; split-wave
# priority; wave clocks and levels segments.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04j}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants r04i,default,prio --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-$c-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants r04i,default,prio --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-b-fail; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 > gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-fail; tail gpurun_out/wclk_$tag.log; exit 1; }
timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 --async-frames >> gpurun_out/wclk_$tag.log 2>&1 || { echo wclk-async-fail; exit 1; }
echo wclk-ok
for c in C4 C5; do
  timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 --variants seglv \
    >> gpurun_out/seglv_$tag.log 2>&1 || { echo seglv-$c-fail; tail gpurun_out/seglv_$tag.log; exit 1; }
done
echo ALLDONE
