cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/e2etr
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/e2etr -o run -- python3 $R/tools/e2e_probe.py --config C3 --frames 6 ${1:+--flags $1} > $R/gpurun_out/e2etr.log 2>&1 || { echo fail; tail $R/gpurun_out/e2etr.log; exit 1; }
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
ev = []
for r in csv.DictReader(open(R + "/gpurun_out/e2etr/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if "render_kernel" in n: n = "render" + n[n.index("<"):n.index(">") + 1]
    elif "copier" in n: n = "copier"
    else: n = n.split("(")[0][-28:]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
ev.sort()
first = next(i for i, e in enumerate(ev) if e[2] == "copier")
ev = ev[max(0, first - 3):first + 40]
t0 = ev[0][0]
for s, e, n, q in ev:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{q} {n}")
PY
