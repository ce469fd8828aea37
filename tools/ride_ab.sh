# colour riders (gsr_colour_mode 2) vs the fused preprocess: tests, alternating rates
# at C and B, then one C kernel trace per mode (per-kernel durations of one step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_colour.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ride_tests.log 2>&1 || { tail -40 gpurun_out/ride_tests.log; exit 1; }
tail -1 gpurun_out/ride_tests.log
for r in 1 2; do
  for m in 0 2; do
    GSR_COLOUR_APART=$m timeout -k 10 300 python tools/graph_probe.py --configs C B --steps 200 --rounds 1 2>&1 | grep round | sed "s/^/mode $m: /"
  done
done
mkdir -p gpurun_out/rtrace
for m in 0 2; do
  GSR_COLOUR_APART=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rtrace -o C$m -- python3 tools/graph_probe.py --configs C --steps 50 --rounds 1 --graph-only > gpurun_out/rtrace/run$m.log 2>&1 || { tail -20 gpurun_out/rtrace/run$m.log; exit 1; }
  python3 - $m <<'PY'
import csv, sys
m = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/rtrace/C{m}_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "preprocess_fwd" in n]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]["Start_Timestamp"])
print("mode", m, "step", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, "us")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:70]}")
PY
done
