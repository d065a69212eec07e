# PMC passes for one config's trace kernel (one counter group per rocprofv3
# run, --kernel-trace only alongside; MI355X_MICROARCH.md "rocprofv3 PMC slots").
# usage (on the GPU box): [VARIANT=name] bash tools/pmc_round.sh <tag> [config] [bands]
#   VARIANT: measure lib/variants/<name>/librt_mi355.so instead of the default build
#   config: C3 (default) / C2 / C4 / C5; bands: 1 (whole frame, default) or N
#   (row band 0 of N: one rank's share of an N-GPU frame).
# Writes gpurun_out/pmc_<tag>_<config>[_b<N>]/summary.json; copy it to
# profiles/pmc_<config>[_b<N>].json (bench.py reads that name).
set -o pipefail
tag=${1:-cur}
cfg=${2:-C3}
bands=${3:-1}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
sfx=$cfg
band_arg=""
if [ "$bands" -gt 1 ]; then sfx=${cfg}_b$bands; band_arg="--band 0/$bands --rgb32f"; fi
kernel=$(python3 -c "import sys; sys.path.insert(0, '$R'); import bench, _rt_pkg; rt = _rt_pkg.load(); fr = rt.make('$cfg'); \
rows = fr.plane.ResolutionY if $bands == 1 else -(-fr.plane.ResolutionY // (8 * $bands)) * 8; \
print(bench.trace_kernel_name('megakernel', fr.spp, fr.max_bounces, fr.plane.ResolutionX, rows, in_flight=True))") || exit 1
# the timed frames are RT_FLAG_ASYNC on eight streams like bench.py's (frames in flight: the same kernel
# instance as the bench line's — a whole frame's non-split one; the first of them, with no frame beside
# it, runs the split instance and is not counted: the summary keeps the named kernel's dispatches)
frames=24
out=$R/gpurun_out/pmc_${tag}_$sfx${VARIANT:+_$VARIANT}
run() {
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 --output-format csv -d $out/$1 -o run -- \
    python3 $R/tools/probe.py --config $cfg --modes megakernel --frames $frames --variants ${VARIANT:-default} --async-frames --streams 8 \
      $band_arg > $out/$1.log 2>&1
}
mkdir -p $out
echo "pmc $cfg bands $bands kernel '$kernel'"
run A "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ" &&
run B "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_HIT TCC_MISS" &&
run C "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" &&
run D "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM" &&
# a whole frame in flight renders its sky tail in sky_batch_kernel (counted with it)
python $R/tools/pmc_summary.py $out/A $out/B $out/C $out/D --kernel "$kernel" --with sky_batch_kernel --config $cfg --bands $bands \
  --out $out/summary.json > /dev/null && echo pmc-ok
