# graph-mode tests + rates at B and C + a kernel trace of B's replays (per-kernel mean)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -30 gpurun_out/graph_tests.log; exit 1; }
tail -1 gpurun_out/graph_tests.log
timeout -k 10 300 python tools/graph_probe.py --configs B C --steps 300 --rounds 2 --graph-only 2>&1 | grep graph
bash tools/graph_trace.sh > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/gtrace/B_kernel_trace.csv")))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(f"{k:50s} {len(v):5d} {sum(v) / len(v):7.1f} us")
PY
