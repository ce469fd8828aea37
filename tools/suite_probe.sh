# full GPU suite, then graph-form rates at B and C (two rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
tail -1 gpurun_out/suite.log
timeout -k 10 300 python tools/graph_probe.py --configs B C --steps 300 --rounds 2 --graph-only 2>&1 | grep graph
