# rebuild loop with the refit strategy at several rebuild thresholds (RT_REFIT_REBUILD)
set -o pipefail
for lim in 1.05 1.1 1.25 100; do
  for c in C3 C5i; do
    echo "== limit $lim $c"
    RT_REFIT_REBUILD=$lim timeout -k 10 200 python tools/rebuild_bench.py --config $c 2>&1 | grep -v amdgpu || exit 1
  done
done
timeout -k 10 200 python tools/rebuild_bench.py --config C5i --frames 20 2>&1 > /dev/null
