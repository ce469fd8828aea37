# L1 partial sums in render_fwd's epilogue (gsr_l1_mode 1) vs in the backward preparation (0):
# GPU tests of the L1 paths, then replayed C and B step traces per mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_model_path.py tests/test_gpu_graph.py tests/test_gpu_split.py tests/test_forward_one_call.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/l1fwd_tests.log 2>&1 || { tail -40 gpurun_out/l1fwd_tests.log; exit 1; }
tail -1 gpurun_out/l1fwd_tests.log
mkdir -p gpurun_out/strace
for cfg in C B; do
for r in 1 2; do
for m in 0 1; do
  GSR_L1_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/strace -o ${cfg}_l1m$m -- python3 tools/graph_probe.py --configs $cfg --steps 100 --rounds 1 --graph-only > gpurun_out/strace/run_${cfg}_l1m$m.log 2>&1 || { tail -20 gpurun_out/strace/run_${cfg}_l1m$m.log; exit 1; }
  python3 tools/trace_medians.py gpurun_out/strace/${cfg}_l1m${m}_kernel_trace.csv
done
done
done
