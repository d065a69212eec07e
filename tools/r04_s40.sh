# Round-4 GPU session 40: a 1/8 share one frame at a time at the final
# library — interleaved A/B against round 3's base and the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ay}
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants base,default --rounds 8 --frames 12 \
  >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
grep variant gpurun_out/abx_$tag.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands 8 --streams 1 > gpurun_out/sb8s1_$tag.log 2>&1 || { echo sb8s1-fail; exit 1; }
grep '^{' gpurun_out/sb8s1_$tag.log | cut -c1-120
echo ALLDONE
