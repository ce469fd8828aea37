#!/bin/bash
# On the box: time each variant library with short bench runs, round-robin over
# ROUNDS rounds (default 2) so clock drift hits every variant alike.
#   ROUNDS=3 bash tools/run_variants.sh base A B ...
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    lib=$PWD/3dgs_study_amd/lib/libgsr_$v.so
    [ "$v" = base ] && lib=$PWD/3dgs_study_amd/lib/libgsr.so
    GSR_LIBRARY=$lib timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --full-steps 0 --exchange-steps 0 --footprint-steps 0 --glue-steps 0 \
        > gpurun_out/var_${v}_$r.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_${v}_$r.log; exit 1; }
    python - "$v" gpurun_out/var_${v}_$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d["stages_ms"]
e = d.get("config_E_render") or {}
es = " E %.1f fps (%s)" % (e["value"], " ".join(f"{k[:5]}={v * 1e3:.0f}" for k, v in e["stages_ms"].items())) if e else ""
b = d.get("config_B") or {}
bs = " B %.1f (%s; depth=%.1f)" % (b["value"], b.get("form"), b["stages_ms"]["depth_sort"] * 1e3) if b else ""
print(f"{sys.argv[1]:>10} {d['value']:8.2f}  " + " ".join(f"{k[:8]}={v * 1e3:.0f}" for k, v in s.items() if v) + es + bs)
PY
  done
done
