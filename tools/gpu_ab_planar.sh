#!/bin/bash
# On the box: parity tests touching the backward layouts, then the dsh layout A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider -x --timeout 300 --timeout-method thread -k "forward_backward_parity or multiview or config_c or python_branch or scale_modifier or empty" > gpurun_out/x7_tests.log 2>&1 || { tail -40 gpurun_out/x7_tests.log; exit 1; }
tail -3 gpurun_out/x7_tests.log
timeout -k 10 300 python -u tools/ab_planar.py > gpurun_out/x7_ab.log 2>&1 || { tail -20 gpurun_out/x7_ab.log; exit 1; }
tail -1 gpurun_out/x7_ab.log
