set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ctrace
GSR_COLOUR_APART=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ctrace -o B -- python3 tools/graph_probe.py --configs B --steps 50 --rounds 1 --graph-only > gpurun_out/ctrace/run.log 2>&1 || { tail -20 gpurun_out/ctrace/run.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/ctrace/B_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "preprocess_fwd" in n]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']} s{r['Stream_Id']}  {r['Kernel_Name'][:60]}")
PY
