#!/bin/bash
# PMC passes over the gsr kernels matching a regex (one rocprofv3 run per counter
# group, no tracing domains mixed with --pmc).  On the box:
#   REGEX='rowspan|rank_gather' bash tools/pmc_kernels.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-pmck}
shift
OUT=/tmp/$TAG
mkdir -p $OUT gpurun_out
export TMPDIR=/tmp
REGEX=${REGEX:-gsr::}
CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --render-steps 0 --footprint-steps 0 --exchange-steps 0 --glue-steps 0 --config-b-steps 0 $*"
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT /tmp/${TAG}_summary.json > gpurun_out/${TAG}_pmc.txt
cat gpurun_out/${TAG}_pmc.txt
