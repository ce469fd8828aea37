#!/bin/bash
# Build experimental variants of one kernel source with -D flags (in this container):
#   bash tools/variants.sh render_bwd "A:-DFOO" "B:-DBAR" ...
# -> 3dgs_study_amd/lib/libgsr_<name>.so ; then on the box:
#   for v in A B; do GSR_LIBRARY=$PWD/3dgs_study_amd/lib/libgsr_$v.so python bench.py ...; done
set -e
SRC=$1; shift
cd "$(dirname "$0")/../3dgs_study_amd/csrc"
make -s
OBJS=""
for f in preprocess binning render_fwd render_bwd preprocess_bwd abi; do
  [ "$f" != "$SRC" ] && OBJS="$OBJS ../build/$f.o"
done
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I../../include -munsafe-fp-atomics \
      -fno-slp-vectorize $flags -c $SRC.hip -o ../build/${SRC}_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/${SRC}_$name.o -o ../lib/libgsr_$name.so
  echo "built libgsr_$name.so ($flags)"
done
