# Library variants (lib/variants/<name>, built by `make VARIANT=<name> EXTRA=…`)
# against the default build: alternating 200-frame bench lines per config.
#   VARIANTS="default lvh6 lvh8" CONFIGS="C5" ROUNDS=2 TAG=r08g bash tools/exp/variant_ab.sh
# Lines -> gpurun_out/vab_${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r08g}
out=gpurun_out/vab_${TAG}.jsonl
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-C5}; do
    for v in ${VARIANTS:-default}; do
      lib=""; [ "$v" != default ] && lib="--lib $v"
      log=gpurun_out/vab_${TAG}_${v}_${c}_$r.log
      timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline --moving-frames 0 $lib \
        > $log 2>&1 || { echo "FAIL $v $c $r"; tail -n 20 $log; exit 1; }
      grep '^{' $log | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'v':'$v','cfg':'$c','r':$r,'value':round(d['value']),'ms':round(d['ms_per_step'],5),'kms':round(d['config']['kernel_ms_per_frame'],5),'canon':d['roofline'].get('canonical_counts',{}).get('state')}))" | tee -a $out
    done
  done
done
