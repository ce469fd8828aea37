# the depth sort's key base published from preprocess's per-workgroup key ranges
# (GSR_PUBLISH_BASE=1) vs reduced by every first-pass downsweep block: binning parity
# tests, then replayed C / B traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_forward_one_call.py tests/test_gpu_graph.py tests/test_model_path.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pb_tests.log 2>&1 || { tail -30 gpurun_out/pb_tests.log; exit 1; }
tail -1 gpurun_out/pb_tests.log
bash tools/step_trace.sh C base:0 nopb:0 base:0 nopb:0 || exit 1
bash tools/step_trace.sh B base:0 nopb:0 || exit 1
