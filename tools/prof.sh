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
python3 tools/prof_summary.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_kernel_stats.csv --top 28
exit $rc
