#!/bin/bash
# One GPU round-trip: parity tests, then the benchmark (no CPU baseline).
# usage (on the box): bash tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest tests/ -q -m gpu -p no:cacheprovider -x -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
else
  timeout -k 10 600 python -m pytest tests/ -q -m gpu -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
fi
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
grep '"metric"' gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
exit $rc
