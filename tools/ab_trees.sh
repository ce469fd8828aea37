#!/bin/bash
# A/B of whole source trees on one box: _var/<name> are git worktrees of other
# commits, each with its own built libgsr.so; every tree runs its own bench.py,
# round-robin over ROUNDS rounds, no stage events in the timed region.
#   ROUNDS=3 bash tools/ab_trees.sh T0 T1 ...   ("." = this tree)
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-300}
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    d=_var/$v; [ "$v" = . ] && d=.
    ( cd $d && B=""; grep -q config-b-steps bench.py && B="--config-b-steps 0"
      timeout -k 10 300 python bench.py --steps $STEPS --warmup 30 --no-cpu-baseline --full-steps 0 \
        --exchange-steps 0 --footprint-steps 0 --glue-steps 0 --render-steps 0 $B \
        --stage-events none ${AB_ARGS:-} ) > gpurun_out/ab_${v//\//_}_$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_${v//\//_}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(f\"{sys.argv[2]:>6} r$r {d['value']:9.2f} it/s {d['ms_per_step']:.4f} ms\")" gpurun_out/ab_${v//\//_}_$r.log "$v"
  done
done
