# Frame-queue shape against hardware queues, alternating lines of the
# driver's window (--steps 20 --warmup 5) and of 200 frames.  A kernel trace
# of the default (r08b: eight streams, GPU_MAX_HW_QUEUES=8) put the eight
# bench streams on five hardware queues (the library's and torch's own
# streams hold the others), so three queues ran two frames back to back.
# Variants: "streams:hwqueues".  Lines -> gpurun_out/queues_${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r08d}
out=gpurun_out/queues_${TAG}.jsonl
line() {  # variant steps rep
  local v=$1 s=$2 r=$3 st=${1%%:*} hq=${1##*:} log=gpurun_out/queues_${1/:/_}_${2}_${3}.log
  timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --moving-frames 0 --streams $st --hw-queues $hq \
    > $log 2>&1 || { echo "FAIL $v $s $r"; tail -n 20 $log; exit 1; }
  grep '^{' $log | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','steps':$s,'r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5),'kms':round(d['config']['kernel_ms_per_frame'],5)}))" | tee -a $out
}
for r in 1 2 3; do
  for v in ${VARIANTS:-8:8 5:8 6:8 8:11 6:11}; do line $v 20 $r || exit 1; done
done
for r in 1 2; do
  for v in ${VARIANTS:-8:8 5:8 6:8 8:11 6:11}; do line $v 200 $r || exit 1; done
done
