# Round-4 GPU session 27 (round-5 groundwork): the one-sample split-wave
# build merged onto the final round-4 library (s64m) — GPU suite, A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r04ag}
RT_TEST_LIB_VARIANT=s64m timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread \
  > gpurun_out/tests_s64m_$tag.log 2>&1 || { echo s64m-suite-fail; tail -60 gpurun_out/tests_s64m_$tag.log; exit 1; }
tail -1 gpurun_out/tests_s64m_$tag.log
for b in 0/8 0/4 0/2; do
  timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants default,s64m --rounds 8 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
for c in C3 C2; do
  timeout -k 10 300 python tools/abx.py --config $c --variants default,s64m --rounds 6 --frames 12 \
    >> gpurun_out/abx_$tag.log 2>&1 || { echo abx-fail; tail gpurun_out/abx_$tag.log; exit 1; }
done
grep variant gpurun_out/abx_$tag.log
for n in 8 4; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --sim-bands $n > gpurun_out/sb${n}_def_$tag.log 2>&1 || { echo sb-fail; exit 1; }
  grep '^{' gpurun_out/sb${n}_def_$tag.log | cut -c1-160
done
echo ALLDONE
