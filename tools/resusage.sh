# Register / spill / scratch use of the render kernels for a set of -D flags.
# usage: bash tools/resusage.sh [file.hip] [extra flags...]
cd "$(dirname "$0")/../unity-raytracer_amd"
f=${1:-trace}; shift
sched=""
[ "$f" = trace ] && sched="-mllvm -amdgpu-sched-strategy=max-memory-clause"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  $sched "$@" --offload-device-only -c -Rpass-analysis=kernel-resource-usage -o /dev/null csrc/$f.hip 2>&1 |
  grep -E 'Function Name|VGPRs:|SGPRs:|Spill|ScratchSize|Occupancy' | sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' |
  paste - - - - - - - | grep -E 'render_(levels_)?kernel' |
  sed -e 's/Function Name: _ZN12_GLOBAL__N_1//' -e 's/EvN3rtd8SceneDevENS1_8FrameDevE//' -e 's/\[bytes\/lane\]//' |
  awk -F'\t' '{printf "%-40s", $1; for (i=2;i<=NF;i++) printf " %s", $i; printf "\n"}'
