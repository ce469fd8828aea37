# full GPU suite + the driver's bench command + a default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench_k20.log 2>&1 || { tail -20 gpurun_out/final_bench_k20.log; exit 1; }
grep '"metric"' gpurun_out/final_bench_k20.log | cut -c1-400
