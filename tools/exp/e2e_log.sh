# e2e rt_render vs slab count and host threads
set -o pipefail
for t in 4 8 12; do
  echo "== threads $t"
  RT_HOST_THREADS=$t timeout -k 10 200 python3 tools/exp/e2e_sweep.py C3 2>&1 | grep -v amdgpu || exit 1
done
