# whole-frame bench lines, library variants alternated
for r in 1 2 3; do
  for v in ${BAB_VARIANTS:-nosky default sky16}; do
    lib=""; [ "$v" != default ] && lib="--lib $v"
    timeout -k 10 200 python bench.py --steps ${BAB_STEPS:-200} --warmup 5 --no-cpu-baseline --moving-frames 0 ${BAB_ARGS:-} $lib > gpurun_out/bab_${v}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/bab_${v}_$r.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5),'kms':round(d['config']['kernel_ms_per_frame'],5),'lone':round(d['config']['lone_kernel_ms_per_frame'],5),'launch':d['config'].get('timed_launch')}))" >> gpurun_out/bab_${BAB_TAG:-r05t}.jsonl
  done
done
