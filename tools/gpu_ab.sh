#!/bin/bash
# One GPU call: the parity tests (minus the slow full-size E test), then an A/B of
# variant libraries.  usage (on the box): bash tools/gpu_ab.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -x -k "not config_e" --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
if [ $# -gt 0 ]; then ROUNDS=${ROUNDS:-2} bash tools/run_variants.sh "$@"; fi
