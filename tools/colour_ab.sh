# colour half apart (gsr_colour_mode) vs fused: tests, then alternating rates at C and B (graph and eager)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_colour.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/colour_tests.log 2>&1 || { tail -40 gpurun_out/colour_tests.log; exit 1; }
tail -1 gpurun_out/colour_tests.log
for r in 1 2; do
  for m in 0 1; do
    GSR_COLOUR_APART=$m timeout -k 10 300 python tools/graph_probe.py --configs C B --steps 200 --rounds 1 2>&1 | grep round | sed "s/^/apart $m: /"
  done
done
