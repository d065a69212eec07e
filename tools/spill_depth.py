"""Scratch (spill / private-array) instructions of a kernel by loop depth,
from the LLVM assembly's block comments.  usage:
    python tools/spill_depth.py <file.s> <kernel-name-substring>"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and name in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
depth, hdr = 0, ""
stats = {}
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):.*", l)
    if m:
        d = re.search(r"Depth=(\d+)", l)
        depth = int(d.group(1)) if d else 0
        h = re.search(r"Header=(\S+)", l)
        hdr = h.group(1) if h else (m.group(1) if "Loop Header" in l else "")
        continue
    s = l.strip()
    if s.startswith("scratch_") or (s.startswith("buffer_") and "off" in s and "s[0:3]" in s):
        kind = "store" if "store" in s else "load"
        key = (depth, kind)
        stats[key] = stats.get(key, 0) + 1
for k in sorted(stats):
    print(f"depth {k[0]} {k[1]:5s} {stats[k]}")
