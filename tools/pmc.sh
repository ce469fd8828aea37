#!/bin/bash
# PMC passes over the benchmark's gsr kernels (one rocprofv3 run per pass, no
# tracing domains mixed with --pmc).  usage (on the box): bash tools/pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
OUT=/tmp/$TAG  # raw CSVs stay on the box; the summary returns
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --render-steps 0 --footprint-steps 0 --exchange-steps 0 --glue-steps 0 --config-b-steps 0 ${PMC_ARGS:-}"
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "gsr::" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
done
mkdir -p gpurun_out
python3 tools/pmc_summary.py $OUT gpurun_out/${TAG}_pmc_summary.json ${PMC_SUFFIX:-} > gpurun_out/${TAG}_pmc${PMC_TXT:-}.txt
cat gpurun_out/${TAG}_pmc${PMC_TXT:-}.txt
