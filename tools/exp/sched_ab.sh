# Machine-scheduler strategies of the two trace files, alternating bench lines
# (library variants built by `make VARIANT=… TRACE_FLAGS=… / LEVELS_FLAGS=…`).
# C3: trace.hip (default max-memory-clause) against max-ilp / GCN default /
# iterative-ilp; C4, C5: trace_levels.hip (default GCN) against
# max-memory-clause / max-ilp.  Lines -> gpurun_out/sched_${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r08a}
out=gpurun_out/sched_${TAG}.jsonl
line() {  # variant config rep
  local v=$1 c=$2 r=$3 lib=""
  [ "$v" != default ] && lib="--lib $v"
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline --moving-frames 0 $lib \
    > gpurun_out/sched_${v}_${c}_$r.log 2>&1 || { echo "FAIL $v $c $r"; tail -n 20 gpurun_out/sched_${v}_${c}_$r.log; exit 1; }
  grep '^{' gpurun_out/sched_${v}_${c}_$r.log | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','cfg':'$c','r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5),'kms':round(d['config']['kernel_ms_per_frame'],5),'lone':round(d['config']['lone_kernel_ms_per_frame'],5),'canon':d['roofline'].get('canonical_counts')}))" | tee -a $out
}
for r in 1 2 3; do
  for v in default t_ilp t_gcn t_iilp; do line $v C3 $r || exit 1; done
done
for r in 1 2; do
  for c in C4 C5; do
    for v in default l_mmc l_ilp; do line $v $c $r || exit 1; done
  done
done
