# Round-4 GPU session 15: frames in flight (streams) for one rank's share and
# the whole frame — the shard's time per stream is its slowest chain under
# load, so more streams may lift a rank's throughput.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04q}
export GPU_MAX_HW_QUEUES=16
for cfg in "8 4" "8 6" "8 8" "8 12" "4 4" "4 8" "2 4" "2 8" "1 4" "1 8"; do
  set -- $cfg
  n=$1; s=$2
  if [ $n -gt 1 ]; then sb="--sim-bands $n"; else sb="--moving-frames 0"; fi
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline $sb --streams $s > gpurun_out/st_${n}_${s}_$tag.log 2>&1 || { echo st-$n-$s-fail; tail gpurun_out/st_${n}_${s}_$tag.log; exit 1; }
  grep '^{' gpurun_out/st_${n}_${s}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', $n, 'streams', $s, round(d['value']), round(d['ms_per_step'],4))"
done
echo ALLDONE
