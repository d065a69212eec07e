"""Host SAH tree vs device LBVH tree for one config: 4-wide SAH cost of the
exported trees (node/leaf surface areas relative to the root), node and leaf
counts, and the kernel's traversal counts of a RT_FLAG_COUNT_TESTS frame."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa
import torch  # noqa
import _rt_pkg
rt = _rt_pkg.load()
name = sys.argv[1] if len(sys.argv) > 1 else "C3"
fr = rt.make(name)
ctx = rt.Context()


def sah(nodes):
    nd = np.frombuffer(nodes.tobytes(), np.float32).reshape(-1, 32)
    ch = nd[:, 24:28].view(np.int32)
    lo = np.stack([nd[:, 0:4], nd[:, 8:12], nd[:, 16:20]], -1)   # lox, loy, loz (node, slot, axis)
    hi = np.stack([nd[:, 4:8], nd[:, 12:16], nd[:, 20:24]], -1)
    valid = np.isfinite(lo).all(-1) & np.isfinite(hi).all(-1)
    d = np.where(valid[..., None], hi - lo, 0.0)
    area = d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0]
    rlo, rhi = lo[0][valid[0]].min(0), hi[0][valid[0]].max(0)
    rd = rhi - rlo
    root = rd[0] * rd[1] + rd[1] * rd[2] + rd[2] * rd[0]
    inner = valid & (ch >= 0)
    leaf = valid & (ch < 0)
    cnt = ((~ch >> 27) & 3) + 1
    # cost: 1 per 4-wide node visit (its 4 box tests) + 1 per primitive test
    c_node = 1.0 + area[inner].sum() / root
    c_prim = (area[leaf] * cnt[leaf]).sum() / root
    # depth of every leaf slot (root 0), BFS
    depth = np.zeros(len(nd), np.int32)
    order = [0]
    leaf_depths = []
    for x in order:
        for c in ch[x]:
            if c >= 0:
                depth[c] = depth[x] + 1
                order.append(int(c))
        leaf_depths += [depth[x] + 1] * int((leaf[x]).sum())
    ld = np.array(leaf_depths)
    return {"nodes": int(len(nd)), "max_depth": int(ld.max()), "mean_leaf_depth": round(float(ld.mean()), 2), "leaves": int(leaf.sum()), "prims_per_leaf": round(float(cnt[leaf].mean()), 3),
            "sah_nodes": round(float(c_node), 2), "sah_prims": round(float(c_prim), 2),
            "sah": round(float(c_node + c_prim), 2)}


for build in (0, 1):
    ctx.set_scene(fr.scene, build)
    q = sah(ctx.export_bvh()[0])
    _, st = ctx.render(fr.camera, fr.plane, rt.frame_params(fr, flags=rt.abi.RT_FLAG_COUNT_TESTS))
    q.update({"build": ["sah_host", "lbvh"][build], "box_tests": st.box_tests, "tri_tests": st.triangle_tests,
              "sph_tests": st.sphere_tests})
    out = torch.empty((fr.plane.ResolutionY, fr.plane.ResolutionX, 4), dtype=torch.float32, device="cuda")
    for label, fl in (("lpt", 0), ("row_order", rt.abi.RT_FLAG_ROW_ORDER)):
        ks = []
        for _ in range(20):
            s2 = ctx.render_device(fr.camera, fr.plane, rt.frame_params(fr, flags=fl), out.data_ptr(), out.numel() * 4)
            ks.append(s2.kernel_ms)
        q["kernel_ms_" + label] = round(float(np.median(ks[4:])), 4)
    print(json.dumps({"config": name, **q}), flush=True)
