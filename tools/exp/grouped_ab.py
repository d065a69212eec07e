"""A/B of an XCD-grouped longest-first order against the plain one (the
RT_LPT_GROUPED switch of that experiment is removed: grouped was +3 % on C3,
profiles/r03_kernel/xcd_grouped_lpt_ab.jsonl).  Two contexts, interleaved rounds of frames
(render_device, single stream), median kernel ms per arm; frames compared
bit for bit."""
import json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa
import _rt_pkg
rt = _rt_pkg.load()
for name in sys.argv[1:] or ["C3", "C2"]:
    fr = rt.make(name)
    outs = [torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    ctxs = [rt.Context(), rt.Context()]
    for c in ctxs:
        c.set_scene(fr.scene)
    p = rt.frame_params(fr)
    ks = [[], []]
    for rnd in range(10):
        for arm in (0, 1):
            os.environ["RT_LPT_GROUPED"] = str(arm)
            for f in range(33):
                st = ctxs[arm].render_device(fr.camera, fr.plane, p, outs[arm].data_ptr(), outs[arm].numel() * 4)
                if rnd >= 1:
                    ks[arm].append(st.kernel_ms)
    torch.cuda.synchronize()
    same = bool(torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)))
    print(json.dumps({"config": name, "plain_ms": round(statistics.median(ks[0]), 4),
                      "grouped_ms": round(statistics.median(ks[1]), 4),
                      "plain_p10": round(sorted(ks[0])[len(ks[0]) // 10], 4),
                      "grouped_p10": round(sorted(ks[1])[len(ks[1]) // 10], 4), "bit_identical": same}), flush=True)
    for c in ctxs:
        c.close()
