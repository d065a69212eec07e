# rt_render end to end (tools/e2e_probe.py), slab-weight variants alternated
for r in 1 2 3; do
  for v in ${E2E_VARIANTS:-default}; do
    for fl in 8 0; do
      timeout -k 10 200 python tools/e2e_probe.py --config C3 --frames 12 --flags $fl --variant $v 2>/dev/null | grep '^{' >> gpurun_out/e2eab_${E2E_TAG:-x}.jsonl || exit 1
    done
  done
done
