cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/e2e3.log
for v in ${1:-default}; do for f in 0 8; do
  timeout -k 10 100 python tools/e2e_probe.py --config C3 --frames 20 --variant $v --flags $f >> gpurun_out/e2e3.log 2>&1 || { echo fail $v; tail -5 gpurun_out/e2e3.log; exit 1; }; done
done
grep -v amdgpu.ids gpurun_out/e2e3.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['variant'], d['flags'], {k: v for k, v in d.items() if 'registered' in k or k in ('kernel_ms','render_pageable_ms')})"
