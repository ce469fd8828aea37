set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "render_bwd|quad_order" --output-format csv -d /tmp/pb1 -o p -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --render-steps 0 > gpurun_out/pb1.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
from collections import defaultdict
v = defaultdict(list)
for f in glob.glob("/tmp/pb1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, x in v.items(): print(k, "FETCH_SIZE KB mean", sum(x) / len(x))
PY
