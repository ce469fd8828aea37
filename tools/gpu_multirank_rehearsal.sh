#!/bin/bash
# On a 1-GPU box: targeted GPU tests, a short N=1 bench, and the N=2 bench path
# rehearsed with gloo (two ranks sharing the GPU) for both gradient exchanges.
# usage (on the box): bash tools/gpu_multirank_rehearsal.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider -x --timeout 300 --timeout-method thread -k "config_e or depth_sort or config_c or multiview" > gpurun_out/x6_tests.log 2>&1 || { tail -30 gpurun_out/x6_tests.log; exit 1; }
tail -3 gpurun_out/x6_tests.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --full-steps 0 > gpurun_out/x6_bench1.log 2>&1 || { tail -20 gpurun_out/x6_bench1.log; exit 1; }
grep '"metric"' gpurun_out/x6_bench1.log | cut -c1-300
for ex in sh-colour allreduce; do
GSR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --grad-exchange $ex > gpurun_out/x6_bench2_$ex.log 2>&1 || { tail -30 gpurun_out/x6_bench2_$ex.log; exit 1; }
grep '"metric"' gpurun_out/x6_bench2_$ex.log | cut -c1-900
done
