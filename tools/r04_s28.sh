# Round-4 GPU session 28: one rank's share with frames in flight, the final
# build against the previous one (prev = 0ba5215), alternating on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ai}
for n in 8 4; do
  for r in 1 2; do
    for v in default prev; do
      a=""; [ $v = prev ] && a="--lib prev"
      timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sim-bands $n $a > gpurun_out/ab_sb${n}_${v}_${r}_$tag.log 2>&1 || { echo sb-fail; exit 1; }
      grep '^{' gpurun_out/ab_sb${n}_${v}_${r}_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', $n, '$v', $r, round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_kernel_ms'],4))"
    done
  done
done
echo ALLDONE
