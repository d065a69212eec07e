for r in 1 2; do
for cfg in "4 8" "6 8" "8 8" "8 16" "12 16"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python bench.py --steps 400 --warmup 10 --no-cpu-baseline --sim-bands 8 --streams $1 > gpurun_out/st_$1_$2_$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/st_$1_$2_$r.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'streams':$1,'queues':$2,'r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5)}))"
done
done
