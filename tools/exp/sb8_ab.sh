# A/B of one rank's 1/8 share (bench --sim-bands 8, twice) and of the full
# frame for library variants built beforehand with
#   make -C unity-raytracer_amd VARIANT=<name> ...   (here: "sorted" = any-hit
# packets with the wave-wide sort, "hyb" = sorted only in the split instance)
set -o pipefail
cd $GRAFT_REPO_ROOT
for k in 1 2; do
for v in default sorted hyb; do
L=""; [ $v != default ] && L="--lib $v"
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands 8 $L > gpurun_out/sbx_${v}_$k.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/sbx_${v}_$k.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', $k, round(d['value']), d['ms_per_step'])"
done; done
for v in default hyb; do
L=""; [ $v != default ] && L="--lib $v"
timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline $L > gpurun_out/fx_${v}.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/fx_${v}.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('full', '$v', round(d['value']), d['ms_per_step'])"
done
