#!/bin/bash
# Kernel-trace statistics of a short benchmark run (on the box).
# usage: bash tools/prof.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-prof}
shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
# raw traces stay in /tmp (they exceed what gpurun copies back); only the summary returns
RAW=/tmp/${TAG}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$RAW" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --full-steps 0 --render-steps 0 --footprint-steps 0 --exchange-steps 0 --glue-steps 0 --config-b-steps 0 "$@" \
    > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
python3 tools/prof_summary.py "$RAW" gpurun_out/${TAG}_kernel_stats.csv --top 40 --step-trace gpurun_out/${TAG}_step_trace.csv
f=$(find "$RAW" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/${TAG}_rocprof_kernel_stats.csv
exit $rc
