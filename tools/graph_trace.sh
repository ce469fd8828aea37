set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gtrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtrace -o B -- python3 tools/graph_probe.py --configs B --steps 100 --rounds 1 --graph-only > gpurun_out/gtrace/run.log 2>&1 || { tail -20 gpurun_out/gtrace/run.log; exit 1; }
find gpurun_out/gtrace -name "*kernel_stats.csv" -o -name "*kernel_trace.csv" | head
