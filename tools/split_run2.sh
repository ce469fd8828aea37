set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split_gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/split_gpu_suite.log; exit 1; }
tail -3 gpurun_out/split_gpu_suite.log
for m in 128 256 0 128 256 0; do
  GSR_SPLIT=$m timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --footprint-steps 0 --exchange-steps 0 --glue-steps 0 --render-steps 0 --full-steps 0 > gpurun_out/split_bench_$m.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/split_bench_$m.log; exit 1; }
  python3 - "$m" <<'PY'
import json,sys
for l in open(f"gpurun_out/split_bench_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d=json.loads(l); b=d["config_B"]
        print("split", sys.argv[1], "B", b["value"], {k: round(v*1e3,1) for k,v in b["stages_ms"].items()}, "host", b["host_ms_per_step"], "wait", b.get("host_wait_ms_per_step"), "busy", b.get("host_busy_ms_per_step"), "raster", b["raster_ms"])
PY
done
