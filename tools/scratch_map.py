"""Scratch (spill / private-array) instructions of one kernel, grouped by the
source line they belong to (build with -gline-tables-only) and loop depth.
usage: python tools/scratch_map.py <file.s> <kernel-name-substring> [--min 1]"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        files[m.group(1)] = m.group(3).split("/")[-1]
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and name in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
loc, depth, out = "?", 0, {}
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):(.*)", l)
    if m:
        d = re.search(r"Depth=(\d+)", m.group(2))
        depth = int(d.group(1)) if d else 0
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    s = l.strip()
    if s.startswith("scratch_"):
        k = (depth, loc)
        out.setdefault(k, [0, 0])[0 if "store" in s else 1] += 1
tot = [0, 0]
for (d, loc), (st, ld) in sorted(out.items()):
    print(f"depth {d}  {loc:28s} store {st:3d} load {ld:3d}")
    tot[0] += st
    tot[1] += ld
print(f"total store {tot[0]} load {tot[1]}")
