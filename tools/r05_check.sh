#!/bin/bash
# Round 5 GPU check: the one-call forward's tests + the parity core, then a bench line.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_forward_one_call.py tests/test_gpu_parity.py tests/test_model_path.py tests/test_poisoned_scratch.py \
    -m "gpu and not slow" > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --full-steps 0 --exchange-steps 0 > gpurun_out/${T}_bench.log 2>&1
rc=$?
grep '"metric"' gpurun_out/${T}_bench.log | cut -c1-600
exit $rc
