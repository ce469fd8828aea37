# XCD bands (GSR_XCD_BANDS=1) vs strips: blend parity tests on the band library, then
# replayed C / B / E traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_LIBRARY=$PWD/3dgs_study_amd/lib/libgsr_band.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_forward_one_call.py tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not full" > gpurun_out/band_tests.log 2>&1 || { tail -30 gpurun_out/band_tests.log; exit 1; }
tail -1 gpurun_out/band_tests.log
bash tools/step_trace.sh C base:0 band:0 base:0 band:0 || exit 1
bash tools/step_trace.sh B base:0 band:0 || exit 1
