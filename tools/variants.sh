#!/bin/bash
# Build experimental variants of the library with -D flags (in this container):
#   bash tools/variants.sh SRC "A:-DFOO" "B:-DBAR" ...
# SRC = one kernel source (render_bwd, ...) or "all" to rebuild every source.
# -> 3dgs_study_amd/lib/libgsr_<name>.so ; time them on the box with
#   bash tools/run_variants.sh base A B
set -e
SRC=$1; shift
cd "$(dirname "$0")/../3dgs_study_amd/csrc"
make -s
ALL="preprocess binning rowspan render_fwd render_bwd preprocess_bwd sh_exchange train_ops knn abi"
mkdir -p ../build/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  OBJS=""
  for f in $ALL; do
    if [ "$SRC" = all ] || [ "$f" = "$SRC" ]; then
      extra=""  # the Makefile's per-object flags
      case $f in render_fwd|render_bwd) extra="-mllvm --amdgpu-sched-strategy=iterative-ilp" ;; esac
      /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I../../include -munsafe-fp-atomics \
          -fno-slp-vectorize $extra $flags -c $f.hip -o ../build/var/${f}_$name.o
      OBJS="$OBJS ../build/var/${f}_$name.o"
    else
      OBJS="$OBJS ../build/$f.o"
    fi
  done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o ../lib/libgsr_$name.so
  echo "built libgsr_$name.so ($flags)"
done
