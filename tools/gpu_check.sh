#!/bin/bash
# One GPU round-trip: parity tests (fast, then the full-size slow ones), the
# benchmark (no CPU baseline) in between.
# usage (on the box): bash tools/gpu_check.sh TAG [pytest -k expr] [slow: 0|1]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
SLOW=${3:-1}
mkdir -p gpurun_out
PYT=(python -u -m pytest tests/ -v -p no:cacheprovider -x --timeout 120 --timeout-method thread)
if [ -n "$K" ]; then PYT+=(-k "$K"); fi
timeout -k 10 900 "${PYT[@]}" -m "gpu and not slow" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
grep '"metric"' gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
if [ $rc -ne 0 ]; then echo "BENCH FAILED rc=$rc"; exit $rc; fi
if [ "$SLOW" = "1" ]; then
  timeout -k 10 1000 "${PYT[@]}" -m "gpu and slow" > gpurun_out/${TAG}_slow_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_slow_tests.log
fi
exit $rc
