# XCD-locality experiment: row-order dispatch (no longest-first) with tiles
# dealt round-robin over XCDs (default) vs one contiguous eighth of the frame
# per XCD group (variant xstrip); kernel time + L2 hit counters.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/xcd
timeout -k 10 200 python3 $R/tools/probe.py --config C3 --modes rowmajor,megakernel --frames 20 --variants default,xstrip \
  > $R/gpurun_out/xcd/probe.log 2>&1 || { echo probe-fail; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in default xstrip; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT TCC_MISS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv \
    -d $R/gpurun_out/xcd/pmc_$v -o run -- python3 $R/tools/probe.py --config C3 --modes rowmajor --frames 3 --variants $v \
    > $R/gpurun_out/xcd/pmc_$v.log 2>&1 || { echo pmc-fail-$v; exit 1; }
  python3 $R/tools/pmc_summary.py $R/gpurun_out/xcd/pmc_$v --kernel "render_kernel<false, false, false, true>" \
    --out $R/gpurun_out/xcd/pmc_$v.json > /dev/null || exit 1
done
echo XCD-DONE
