# r05h: C4/C5 counters and segment clocks at the LDS-sum build; a 1/8 share's
# one-frame-at-a-time kernel trace (the bench line vs A/B gap)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
PMC_SET="C4:1 C5:1" bash tools/gpu_session.sh r05h pmcall || exit 1
for c in C4 C5; do
  timeout -k 10 300 python tools/probe.py --config $c --modes megakernel --frames 3 --variants seglv,default \
    >> gpurun_out/seglv_r05h.log 2>&1 || { echo seglv-fail; tail gpurun_out/seglv_r05h.log; exit 1; }
done
echo seglv-ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_sb8s1_r05h -o run --output-format csv -- \
  python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands 8 --streams 1 \
  > $R/gpurun_out/kt_sb8s1_r05h.log 2>&1 || { echo kt-sb8-fail; exit 1; }
cd $R
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands 8 --streams 1 \
  > gpurun_out/sb8s1_r05h.log 2>&1 || { echo sb8s1-fail; exit 1; }
timeout -k 10 300 python tools/abx.py --config C3 --band 0/8 --variants default --rounds 6 --frames 12 \
  > gpurun_out/abx_sb8_r05h.log 2>&1 || { echo abx-fail; exit 1; }
echo ALLDONE
