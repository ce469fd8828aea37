#!/bin/bash
# One GPU call of round 4: fast GPU tests, the default bench line, the exchange's
# per-rank cost split (tools/exchange_profile.py), then optional A/B variants.
# usage (on the box): bash tools/r04_check.sh TAG [variant ...]
set -o pipefail
TAG=${1:-r04}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -v -p no:cacheprovider -x --timeout 120 --timeout-method thread \
    -m "gpu and not slow" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python - gpurun_out/${TAG}_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("C", d["value"], d["ms_per_step"], "raster", d.get("raster_ms"), {k: round(v * 1e3, 1) for k, v in d["stages_ms"].items()})
print("exchange_1rank", d.get("exchange_1rank"))
e = d.get("config_E_render") or {}
print("E", e.get("value"), {k: round(v * 1e3, 1) for k, v in e.get("stages_ms", {}).items()})
PY
timeout -k 10 300 python tools/exchange_profile.py --steps 50 --rounds 2 > gpurun_out/${TAG}_exprof.log 2>&1 || { tail -20 gpurun_out/${TAG}_exprof.log; exit 1; }
grep -v "^{" gpurun_out/${TAG}_exprof.log
if [ $# -gt 0 ]; then ROUNDS=2 bash tools/run_variants.sh base "$@"; fi
