#!/bin/bash
# On the box: time the default library under environment variants, round-robin over
# ROUNDS rounds (default 2).  Each variant is NAME=VAR=VALUE[,VAR=VALUE...]; "base"
# runs with no extra variables.
#   ROUNDS=3 bash tools/run_env_variants.sh base nocs=GSR_COLOUR_STREAM=0
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}; vars=""
    [ "$spec" != "$name" ] && vars=$(echo "${spec#*=}" | tr ',' ' ')
    env $vars timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --full-steps 0 --footprint-steps 0 --glue-steps 0 ${BENCH_ARGS:-} \
        > gpurun_out/envvar_${name}_$r.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/envvar_${name}_$r.log; exit 1; }
    python - "$name" gpurun_out/envvar_${name}_$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d["stages_ms"]
e = d.get("config_E_render") or {}
x = d.get("exchange_1rank") or {}
es = " E %.1f fps" % e["value"] if e else ""
xs = " X %.1f (x%.4f)" % (x["value"], x["vs_plain_ms"]) if x else ""
print(f"{sys.argv[1]:>10} {d['value']:8.2f}  " + " ".join(f"{k[:8]}={v * 1e3:.0f}" for k, v in s.items() if v) + es + xs)
PY
  done
done
