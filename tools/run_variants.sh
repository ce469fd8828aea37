#!/bin/bash
# On the box: time each variant library with a short bench run.
#   bash tools/run_variants.sh A B ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=$PWD/3dgs_study_amd/lib/libgsr_$v.so
  [ "$v" = base ] && lib=$PWD/3dgs_study_amd/lib/libgsr.so
  GSR_LIBRARY=$lib timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_$v.log; exit 1; }
  python - "$v" gpurun_out/var_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["stages_ms"])
PY
done
