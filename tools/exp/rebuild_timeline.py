"""Kernels and copies of the last rebuild+frame in rebuild_trace.sh's trace."""
import csv, sys
d = sys.argv[1]
ks = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
cp = list(csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:60]) for k in ks]
ev += [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), "COPY " + c["Direction"][12:]) for c in cp]
ev.sort()
starts = [i for i, e in enumerate(ev) if "k_vertices" in e[2]]
i0 = starts[-2]
i1 = starts[-1]
t0 = ev[i0][0]
prev = t0
for s, e, n in ev[i0:i1]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:6.1f}  {n}")
    prev = e
