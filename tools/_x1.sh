set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python tools/sh_exchange_cost.py > gpurun_out/x1_shx.log 2>&1 || { tail -5 gpurun_out/x1_shx.log; exit 1; }
tail -1 gpurun_out/x1_shx.log
ROUNDS=2 bash tools/run_variants.sh base t32 || exit 1
for r in 1 2; do for ev in none all; do
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --full-steps 0 --footprint-steps 0 --render-steps 0 --stage-events $ev > gpurun_out/x1_ev_${ev}_$r.log 2>&1 || exit 1
  echo "$ev $(grep '"metric"' gpurun_out/x1_ev_${ev}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
