# colour riders A/B over variant libraries: args "lib:mode" (lib base = libgsr.so);
# alternating graph-form rates at C and B, then one C kernel trace per pair
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
libof() { [ "$1" = base ] && echo $PWD/3dgs_study_amd/lib/libgsr.so || echo $PWD/3dgs_study_amd/lib/libgsr_$1.so; }
for r in 1 2; do
  for vm in "$@"; do
    v=${vm%%:*}; m=${vm#*:}
    GSR_LIBRARY=$(libof $v) GSR_COLOUR_APART=$m timeout -k 10 300 python tools/graph_probe.py --configs C B --steps 200 --rounds 1 --graph-only 2>&1 | grep round | sed "s/^/$v mode $m: /"
  done
done
mkdir -p gpurun_out/rtrace
for vm in "$@"; do
  v=${vm%%:*}; m=${vm#*:}
  GSR_LIBRARY=$(libof $v) GSR_COLOUR_APART=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rtrace -o C_${v}_$m -- python3 tools/graph_probe.py --configs C --steps 50 --rounds 1 --graph-only > gpurun_out/rtrace/run_${v}_$m.log 2>&1 || { tail -20 gpurun_out/rtrace/run_${v}_$m.log; exit 1; }
  python3 - C_${v}_$m <<'PY'
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(f"gpurun_out/rtrace/{sys.argv[1]}_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "preprocess_fwd" in n]
# median over the last 30 steps of each position in the step
steps = [(idx[k], idx[k + 1]) for k in range(len(idx) - 31, len(idx) - 1)]
per = defaultdict(list); tot = []
for a, b in steps:
    tot.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    for j, r in enumerate(rows[a:b]):
        per[j].append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:64]))
med = lambda v: sorted(v)[len(v) // 2]
print(sys.argv[1], "step median", med(tot), "us")
for j in sorted(per):
    print(f"  {med([d for d, _ in per[j]]):7.1f}  {per[j][0][1]}")
PY
done
