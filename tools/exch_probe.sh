# does an earlier graph capture slow the one-rank exchange measurement?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
for v in nograph graph; do
  if [ $v = nograph ]; then extra="--graph-steps 0 --config-b-steps 0"; else extra=""; fi
  timeout -k 10 400 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --footprint-steps 0 --glue-steps 0 --render-steps 0 --full-steps 0 $extra > gpurun_out/exch_$v.log 2>&1 || { tail -20 gpurun_out/exch_$v.log; exit 1; }
  python3 - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/exch_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); ex = d["exchange_1rank"]
        print(sys.argv[1], "C", d["value"], d.get("form"), "exchange", ex["value"], ex["ms_per_step"], ex["vs_plain_ms"])
PY
done
done
