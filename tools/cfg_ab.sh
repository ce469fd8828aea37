#!/bin/bash
# On the box: the bench at configs B and C for the default library and one variant
# (libgsr_<V>.so), two alternating rounds; prints the stage times.
#   usage: bash tools/cfg_ab.sh V [CONFIGS]
set -o pipefail
mkdir -p gpurun_out
V=${1:?variant}; CFGS=${2:-"B C"}
for cfg in $CFGS; do for r in 1 2; do for v in base $V; do
  lib=$PWD/3dgs_study_amd/lib/libgsr_$v.so; [ $v = base ] && lib=$PWD/3dgs_study_amd/lib/libgsr.so
  GSR_LIBRARY=$lib timeout -k 10 200 python bench.py --config $cfg --steps 60 --warmup 10 --no-cpu-baseline \
      --full-steps 0 --footprint-steps 0 --render-steps 0 > gpurun_out/cfg_${cfg}_${v}_$r.log 2>&1 \
      || { echo "$v $cfg failed"; tail -3 gpurun_out/cfg_${cfg}_${v}_$r.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], round(d['value'],1), {k: round(v*1e3) for k,v in d['stages_ms'].items()})" gpurun_out/cfg_${cfg}_${v}_$r.log $cfg $v
done; done; done
