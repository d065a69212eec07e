# Round-4 GPU session 39: round-end rehearsal at the committed final library
# and counter files, plus one rank's 1/8 and 1/4 shares one frame at a time.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ax}
bash tools/r04_s34b.sh $tag || exit 1
for n in 8 4; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands $n --streams 1 > gpurun_out/sb${n}s1_$tag.log 2>&1 || { echo sb${n}s1-fail; exit 1; }
  grep '^{' gpurun_out/sb${n}s1_$tag.log | cut -c1-160
done
echo ALLDONE
