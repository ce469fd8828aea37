set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for b in rowspan lsd; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --full-steps 0 --exchange-steps 0 --glue-steps 0 --binning $b > gpurun_out/ab1_${b}_$r.log 2>&1 || { echo "$b failed"; tail -5 gpurun_out/ab1_${b}_$r.log; exit 1; }
  python - $b gpurun_out/ab1_${b}_$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
def f(x): return " ".join(f"{k[:8]}={v*1e3:.1f}" for k, v in x["stages_ms"].items() if v)
print(sys.argv[1], "C", d["value"], f(d))
t = d.get("footprint_tight"); print("  tight", t["value"], f(t))
b = d.get("config_B"); print("  B", b["value"], f(b), "host", b["host_ms_per_step"], "ms", b["ms_per_step"])
for k in ("config_E_render", "config_E_render_tight"):
    e = d.get(k); print("  ", k, e["value"], f(e))
PY
done
done
