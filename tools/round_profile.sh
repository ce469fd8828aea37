#!/bin/bash
# Round deliverables on the box: the default benchmark line (with the CPU
# baseline), the rocprofv3 kernel trace of config C and E, the PMC passes of
# config C and E in both footprints (bench.py keys the PMC records "<stage>_<config>_<footprint>"),
# then the GPU parity tests (all, incl. slow).
# usage: bash tools/round_profile.sh TAG [skip-tests] [skip-bench]
set -o pipefail
TAG=${1:-round}
mkdir -p gpurun_out
if [ "${3:-}" != "skip-bench" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-300
fi
bash tools/prof.sh ${TAG}_C || exit 1
bash tools/prof.sh ${TAG}_E --config E || exit 1
rm -f gpurun_out/${TAG}_pmc_summary.json
PMC_SUFFIX="_C_rect" bash tools/pmc.sh ${TAG} > /dev/null || exit 1
GSR_FOOTPRINT=tight PMC_SUFFIX="_C_tight --merge" PMC_TXT=_C_tight bash tools/pmc.sh ${TAG} > /dev/null || exit 1
PMC_ARGS="--config E" PMC_SUFFIX="_E_rect --merge" PMC_TXT=_E_rect bash tools/pmc.sh ${TAG} > /dev/null || exit 1
GSR_FOOTPRINT=tight PMC_ARGS="--config E" PMC_SUFFIX="_E_tight --merge" PMC_TXT=_E_tight bash tools/pmc.sh ${TAG} > /dev/null || exit 1
echo profiles done
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -4 gpurun_out/${TAG}_tests.log
  exit $rc
fi
