#!/bin/bash
# Kernel-trace statistics of a short benchmark run (on the box).
# usage: bash tools/prof.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-prof}
shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:90]}")
PY
exit $rc
