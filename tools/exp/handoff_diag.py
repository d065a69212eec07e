"""Diagnose test_one_sample_handoff_under_concurrent_streams: four contexts
render lone 1/8 C3 shares (bands 1, 3, 5, 7) concurrently, frame after frame;
each frame is compared with the row-major share and the mismatching pixels are
described (count, rows/cols, values, the context's last launch).
python handoff_diag.py <variant|-> <trials> <mode: conc|seq>"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa
import torch  # noqa
import _rt_pkg
rt = _rt_pkg.load()
if sys.argv[1] != "-":
    rt.abi.LIB_PATH = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", sys.argv[1], "librt_mi355.so")
trials, mode = int(sys.argv[2]), sys.argv[3]
fr = rt.make("C3")
bad = 0
for t in range(trials):
    ctxs, streams, outs, refs = [], [], [], []
    for k in range(4):
        c = rt.Context()
        c.set_scene(fr.scene)
        kw = dict(band_index=2 * k + 1, band_count=8, band_rows=8)
        ref, _ = c.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ROW_ORDER, **kw))
        s = torch.cuda.Stream()
        c.set_stream(s.cuda_stream)
        ctxs.append((c, rt.frame_params(fr, flags=rt.abi.RT_FLAG_ASYNC, **kw)))
        streams.append(s)
        outs.append(torch.empty(ref.shape, dtype=torch.float32, device="cuda"))
        refs.append(ref)
    for f in range(8):
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        for k, (c, p) in enumerate(ctxs):
            c.render_device(fr.camera, fr.plane, p, outs[k].data_ptr(), outs[k].numel() * 4)
            if mode == "seq":
                c.finish()
        if mode != "seq":
            for c, p in ctxs:
                c.finish()
        torch.cuda.synchronize()
        for k, (c, p) in enumerate(ctxs):
            got = outs[k].cpu().numpy()
            d = got.view(np.uint32) != refs[k].view(np.uint32)
            if d.any():
                bad += 1
                ys, xs, cs = np.nonzero(d)
                print(f"t{t} f{f} k{k}: {d.any(axis=2).sum()} pixels differ; rows {sorted(set(ys.tolist()))[:12]} "
                      f"cols {sorted(set(xs.tolist()))[:12]}; nan {int(np.isnan(got).any(axis=2).sum())}", flush=True)
                for y, x in list(dict.fromkeys(zip(ys.tolist(), xs.tolist())))[:4]:
                    print("   ", y, x, got[y, x].tolist(), refs[k][y, x].tolist(), flush=True)
                print("    last_launch:", c.last_launch(), flush=True)
        print(f"t{t} f{f} done; launch k0: {ctxs[0][0].last_launch()}", flush=True)
    for c, _ in ctxs:
        c.set_stream(None)
        c.close()
print("BAD", bad, flush=True)
