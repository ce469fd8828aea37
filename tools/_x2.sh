set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python tools/sh_exchange_cost.py > gpurun_out/x2_shx.log 2>&1 || { tail -5 gpurun_out/x2_shx.log; exit 1; }
tail -1 gpurun_out/x2_shx.log
timeout -k 10 600 python -u -m pytest tests/test_multiview.py -x -q -m "gpu and not slow" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/x2_mv.log 2>&1 || { tail -20 gpurun_out/x2_mv.log; exit 1; }
tail -2 gpurun_out/x2_mv.log
for r in 1 2; do for ev in none split; do
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --full-steps 0 --footprint-steps 0 --render-steps 0 --stage-events $ev > gpurun_out/x2_ev_${ev}_$r.log 2>&1 || exit 1
  echo "$ev $(grep '"metric"' gpurun_out/x2_ev_${ev}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stages_ms"], d["roofline"]["avg_launch_ms"])')"
done; done
timeout -k 10 300 python bench.py --no-cpu-baseline --full-steps 0 > gpurun_out/x2_bench.log 2>&1 || exit 1
grep '"metric"' gpurun_out/x2_bench.log | cut -c1-3000
