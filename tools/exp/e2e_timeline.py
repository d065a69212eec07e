"""Timeline of the last synchronous rt_render frame in an e2e_trace.sh trace:
kernels and memory copies relative to the frame's first render launch, plus
the rtr frame markers (hipEventRecord/hipStreamSynchronize API calls)."""
import csv, sys

d = sys.argv[1]
ks = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
cp = list(csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:40], k["Queue_Id"]) for k in ks]
ev += [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), "COPY " + c["Direction"][12:], "-") for c in cp]
ev.sort()
renders = [e for e in ev if "render" in e[2]]
# frames: group render launches separated by > 300 us
frames, cur = [], [renders[0]]
for e in renders[1:]:
    if e[0] - cur[-1][0] > 300_000:
        frames.append(cur)
        cur = [e]
    else:
        cur.append(e)
frames.append(cur)
f = frames[-2] if len(frames) > 1 else frames[-1]
t0 = f[0][0]
t1 = max(e[1] for e in f) + 900_000
for s, e, n, q in ev:
    if t0 - 50_000 <= s <= t1:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3} {n}")
