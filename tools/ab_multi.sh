#!/bin/bash
# One GPU call: a short parity check of each variant library, then a round-robin
# timing A/B of all of them against the default library.
#   usage (on the box): ROUNDS=3 bash tools/ab_multi.sh VARIANT...
set -o pipefail
mkdir -p gpurun_out
for V in "$@"; do
  timeout -k 5 200 env GSR_LIBRARY=$PWD/3dgs_study_amd/lib/libgsr_$V.so python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu \
      -p no:cacheprovider -k "forward_backward_parity and (cfg1 or cfg2) or needle" --timeout 150 --timeout-method thread \
      > gpurun_out/${V}_par.log 2>&1 || { echo "$V parity failed"; tail -5 gpurun_out/${V}_par.log; exit 1; }
  echo "$V parity: $(tail -1 gpurun_out/${V}_par.log)"
done
ROUNDS=${ROUNDS:-2} bash tools/run_variants.sh base "$@"
