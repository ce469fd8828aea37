#!/bin/bash
# Kernel traces of the exchange variants (tools/exchange_profile.py), one process each,
# plus one untraced pass: where the forced one-rank exchange's extra step time goes.
# usage (on the box): bash tools/exprof_trace.sh TAG [variant ...]
set -o pipefail
TAG=${1:-exprof}; shift
VARS=${*:-plain rccl}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/exchange_profile.py --steps 60 --rounds 2 --no-wrap --only $(echo $VARS | tr ' ' ,) \
    > gpurun_out/${TAG}_untraced.log 2>&1 || { tail -20 gpurun_out/${TAG}_untraced.log; exit 1; }
grep -v "^{" gpurun_out/${TAG}_untraced.log | grep -E "^(plain|local|rccl)"
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  RAW=/tmp/${TAG}_${v}
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv rocpd -d "$RAW" -o run -- \
      python3 "$GRAFT_REPO_ROOT/tools/exchange_profile.py" --steps 30 --rounds 1 --no-wrap --only $v \
      > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_${v}_prof.log" 2>&1 || exit 1
  (cd "$GRAFT_REPO_ROOT" && python3 tools/prof_summary.py "$RAW" gpurun_out/${TAG}_${v}_kernel_stats.csv --top 30 \
      --step-trace gpurun_out/${TAG}_${v}_step_trace.csv > /dev/null) || exit 1
done
