# A lone whole frame's sky batches: none (default: the sky tiles are waves of
# the render launch), after the render launch (skylone, -DRT_EXP_SKYLONE=1) or
# beside it on a second stream (skyside, -DRT_EXP_SKYLONE=2: measured in r08f
# and removed from the sources, 0.241 -> 0.264 ms); alternating
# bench lines (lone_kernel_ms_per_frame: 20 frames back to back on one
# stream; the synchronous rt_render lines), then the variant's parity tests.
# Lines -> gpurun_out/skylone_${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r08f}
out=gpurun_out/skylone_${TAG}.jsonl
line() {  # variant config rep
  local v=$1 c=$2 r=$3 lib="" log=gpurun_out/skylone_${1}_${2}_${3}.log
  [ "$v" != default ] && lib="--lib $v"
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --moving-frames 0 $lib > $log 2>&1 \
    || { echo "FAIL $v $c $r"; tail -n 20 $log; exit 1; }
  grep '^{' $log | tail -n 1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print(json.dumps({'v':'$v','cfg':'$c','r':$r,'value':round(d['value']),'lone':round(c['lone_kernel_ms_per_frame'],5),'lone_launch':c['lone_launch'],'e2e8':round(c.get('end_to_end_rgba8_ms_per_frame') or 0,4),'e2e':round(c.get('end_to_end_ms_per_frame') or 0,4)}))" | tee -a $out
}
for r in 1 2 3; do
  for v in ${VARIANTS:-default skyside skylone}; do line $v C3 $r || exit 1; done
done
for v in ${VARIANTS:-default skyside skylone}; do line $v C2 1 || exit 1; done
if [ -n "${PARITY_VARIANT:-skyside}" ]; then
  RT_TEST_LIB_VARIANT=${PARITY_VARIANT:-skyside} timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_sky.py \
    tests/test_gpu_parity.py -m gpu -k "not sky_count_waits" -x -q --timeout 170 --timeout-method thread > gpurun_out/skylone_parity_${TAG}.log 2>&1 \
    || { echo "parity FAIL"; tail -n 40 gpurun_out/skylone_parity_${TAG}.log; exit 1; }
  tail -n 2 gpurun_out/skylone_parity_${TAG}.log
fi
