"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

    python tools/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB ... --kernel render_kernel --out profiles/pmc_C3.json

HBM bytes (gfx950, MI355X_MICROARCH.md "HBM"): TCC_EA0_RDREQ_{32B,64B,128B}
and TCC_EA0_WRREQ(_64B) count L2 -> fabric requests (Infinity-Cache hits are
counted too, so this is an upper bound on DRAM bytes):
  read  = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (if the split counters
          are present; otherwise 2 * 64 * RDREQ, the guide's wide-read correction)
  write = 64*WRREQ_64B + 32*(WRREQ - WRREQ_64B)
"""
import argparse
import csv
import glob
import hashlib
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(dirs):
    """kernel -> counter -> [per-dispatch values], over the dispatches of the
    kernel's most frequent grid only: the workload's launches, not the tiny
    warm-up frames a context renders at its first rt_set_scene (same kernel
    names), nor a stream's first frame before its longest-first order exists
    (whose whole-frame launch has no sky tail: a larger grid)."""
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            names, grids = {}, {}
            for row in csv.DictReader(open(f)):
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                names[did] = row["Kernel_Name"]
                grids[did] = int(float(row.get("Grid_Size") or 0))
                per[did][row["Counter_Name"]] += float(row["Counter_Value"])
            freq = defaultdict(lambda: defaultdict(int))
            for did, g in grids.items():
                freq[names[did]][g] += 1
            mode = {k: max(v.items(), key=lambda gv: (gv[1], gv[0]))[0] for k, v in freq.items()}
            for did, cs in per.items():
                if grids[did] != mode[names[did]]:
                    continue
                for c, v in cs.items():
                    vals[names[did]][c].append(v)
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="render_kernel<false>")
    ap.add_argument("--with", dest="with_", default="",
                    help="a kernel launched once per frame beside --kernel (sky_batch_kernel): its per-dispatch "
                         "counters are added, the per-frame figures cover both")
    ap.add_argument("--out", default="")
    ap.add_argument("--config", default="", help="recorded: the config the counters were taken on")
    ap.add_argument("--bands", type=int, default=1, help="recorded: row band 0 of N (one rank's share)")
    ap.add_argument("--lib", default=os.path.join(ROOT, "unity-raytracer_amd", "lib", "librt_mi355.so"),
                    help="the library the counters were measured with (its sha256 is recorded; bench.py uses "
                         "the counters only with the same build)")
    a = ap.parse_args()
    vals = load(a.dirs)
    summary = {}
    for k, cs in vals.items():
        summary[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    pick = {k: v for k, v in summary.items() if a.kernel in k}
    res = {"kernels": summary, "config": a.config or None, "bands": a.bands}
    if pick:
        name, c = max(pick.items(), key=lambda kv: len(kv[1]))
        comp = {k: v for k, v in summary.items() if a.with_ and a.with_ in k}
        if comp:
            wname, wc = max(comp.items(), key=lambda kv: len(kv[1]))
            c = {k: c.get(k, 0.0) + wc.get(k, 0.0) for k in set(c) | set(wc)}
            res["with"] = wname
        rd = None
        if "TCC_EA0_RDREQ_32B" in c and "TCC_EA0_RDREQ_64B" in c and "TCC_EA0_RDREQ_128B" in c:
            rd = 32 * c["TCC_EA0_RDREQ_32B"] + 64 * c["TCC_EA0_RDREQ_64B"] + 128 * c["TCC_EA0_RDREQ_128B"]
        elif "TCC_EA0_RDREQ" in c:
            rd = 2 * 64 * c["TCC_EA0_RDREQ"]
        wr = None
        if "TCC_EA0_WRREQ" in c:
            w64 = c.get("TCC_EA0_WRREQ_64B", 0.0)
            wr = 64 * w64 + 32 * (c["TCC_EA0_WRREQ"] - w64)
        res.update({"kernel": name, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                    "hbm_bytes_per_launch": (rd or 0) + (wr or 0) if rd is not None else None,
                    "counters": c})
    if os.path.exists(a.lib):
        h = hashlib.sha256()
        with open(a.lib, "rb") as f:
            h.update(f.read())
        res["lib_sha256"] = h.hexdigest()
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
