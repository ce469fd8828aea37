# per-kernel medians of replayed steps: bash tools/step_trace.sh CONFIG [lib:mode ...]
# (lib base = libgsr.so; mode = gsr_colour_mode)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=$1; shift
libof() { [ "$1" = base ] && echo $PWD/3dgs_study_amd/lib/libgsr.so || echo $PWD/3dgs_study_amd/lib/libgsr_$1.so; }
mkdir -p gpurun_out/strace
for vm in "${@:-base:0}"; do
  v=${vm%%:*}; m=${vm#*:}
  GSR_LIBRARY=$(libof $v) GSR_COLOUR_APART=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/strace -o ${cfg}_${v}_$m -- python3 tools/graph_probe.py --configs $cfg --steps 100 --rounds 1 --graph-only > gpurun_out/strace/run_${cfg}_${v}_$m.log 2>&1 || { tail -20 gpurun_out/strace/run_${cfg}_${v}_$m.log; exit 1; }
  python3 tools/trace_medians.py gpurun_out/strace/${cfg}_${v}_${m}_kernel_trace.csv
done
