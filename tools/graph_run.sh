set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --footprint-steps 0 --exchange-steps 0 --glue-steps 0 --render-steps 0 --full-steps 0 > gpurun_out/graph_bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/graph_bench.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/graph_bench.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print("C", d["value"], d["form"], "eager", d["eager"], "graph", d["graph"], "host", d["host_ms_per_step"])
        b = d["config_B"]
        print("B", b["value"], b["form"], "eager", b["eager"], "graph", b["graph"])
PY
for m in 0 -1 0 -1; do
  GSR_SPLIT=$m timeout -k 10 300 python tools/graph_probe.py --configs B --steps 300 --rounds 2 2>&1 | grep round | sed "s/^/split $m: /"
done
