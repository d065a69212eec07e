# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) against the
# runtime's default, alternating lines of the driver's window
# (--steps 20 --warmup 5) and 200 frames.  Lines -> gpurun_out/kernarg_${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r08c}
out=gpurun_out/kernarg_${TAG}.jsonl
line() {  # env-value steps rep
  local k=$1 s=$2 r=$3 log=gpurun_out/kernarg_${1}_${2}_${3}.log
  if [ "$k" = dev ]; then
    HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --moving-frames 0 > $log 2>&1
  else
    timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --moving-frames 0 > $log 2>&1
  fi || { echo "FAIL $k $s $r"; tail -n 20 $log; exit 1; }
  grep '^{' $log | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'kernarg':'$k','steps':$s,'r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5),'kms':round(d['config']['kernel_ms_per_frame'],5),'lone':round(d['config']['lone_kernel_ms_per_frame'],5),'e2e8':round(d['config']['end_to_end_rgba8_ms_per_frame'],4),'e2e':round(d['config']['end_to_end_ms_per_frame'],4)}))" | tee -a $out
}
for r in 1 2 3; do
  for k in default dev; do line $k 20 $r || exit 1; done
done
for r in 1 2; do
  for k in default dev; do line $k 200 $r || exit 1; done
done
