#!/bin/bash
# One kernel-traced step of the forced one-rank exchange (tools/exchange_profile.py
# rccl variant), printed with its gaps and queues (tools/trace_step.py).
# usage (on the box): bash tools/xtrace.sh TAG
set -o pipefail
TAG=${1:-xtrace}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
RAW=/tmp/${TAG}_rccl
timeout -k 10 300 rocprofv3 --kernel-trace -f rocpd -d "$RAW" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/exchange_profile.py" --steps 30 --rounds 1 --no-wrap --only rccl ${XARGS:-} \
    > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
db=$(find "$RAW" -name "*.db" | head -1)
python3 tools/trace_step.py "$db" --marker render_fwd --index 20 > gpurun_out/${TAG}_step.txt
cat gpurun_out/${TAG}_step.txt
python3 tools/xgaps.py "$db" | tee gpurun_out/${TAG}_gaps.txt
