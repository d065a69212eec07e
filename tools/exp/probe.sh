# usage: bash tools/exp/probe.sh <tag> <variants> <configs> [extra probe args]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; vars=$2; cfgs=$3; shift 3
for c in ${cfgs//,/ }; do
  timeout -k 10 200 python tools/probe.py --config $c --modes megakernel --frames 20 --variants $vars "$@" >> gpurun_out/probe_$tag.log 2>&1 || { echo probe-fail-$c; tail -5 gpurun_out/probe_$tag.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/probe_$tag.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['variant'], d['config'], d['kernel_ms'], d['Mrays_s'], d['same_as_base'], d.get('seg_per_wave',''))
"
