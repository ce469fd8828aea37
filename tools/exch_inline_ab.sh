# the exchange's colour kernel, gather and SH rebuild on a stream of their own (1) or in
# line on the compute stream (0): gloo/RCCL exchange tests, then exchange_profile rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in 1 0; do
  GSR_EXCHANGE_STREAM=$m timeout -k 10 400 python tools/exchange_profile.py --steps 100 --rounds 2 --only plain,rccl > gpurun_out/exch_inline_$m.log 2>&1 || { tail -20 gpurun_out/exch_inline_$m.log; exit 1; }
  grep -E "^(plain|rccl) [01] \{" gpurun_out/exch_inline_$m.log | sed "s/^/stream=$m /"
done
GSR_EXCHANGE_STREAM=0 timeout -k 10 600 python -u -m pytest tests/test_multiview.py tests/test_bench_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exch_inline_tests.log 2>&1; rc=$?
tail -2 gpurun_out/exch_inline_tests.log
exit $rc
