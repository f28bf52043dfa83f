#!/bin/bash
# Build libgs4d with some source files taken from a git revision (default HEAD; WORKTREE = the files as they
# are now) into 4dgaussians-fast-train_amd/build/variant_<name>/libgs4d.so, every other object from the
# current build:
#   tools/build_variant.sh <name> <rev> <csrc file> [<csrc file> ...]
# A/B on the box: LD_LIBRARY_PATH=4dgaussians-fast-train_amd/build/variant_<name> python bench.py ...
# (the bindings' RUNPATH yields to LD_LIBRARY_PATH).
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/4dgaussians-fast-train_amd
OUT=$PKG/build/variant_$NAME
mkdir -p $OUT
BASE="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-result -I$ROOT/include"
for SRC in "$@"; do
  if [ "$REV" = WORKTREE ]; then cp $PKG/csrc/$SRC $PKG/csrc/.variant_$SRC; else git -C $ROOT show $REV:4dgaussians-fast-train_amd/csrc/$SRC > $PKG/csrc/.variant_$SRC; fi
  FLAGS="$BASE"
  case $SRC in preprocess.hip|binning.hip|preprocess_backward.hip|knn.hip|train_tail.hip|hexplane.hip) FLAGS="$FLAGS -ffp-contract=off";; esac
  case $SRC in render.hip) FLAGS="$FLAGS ${RENDER_FLAGS--fno-slp-vectorize -mllvm -amdgpu-sched-strategy=iterative-ilp}";; esac
  case $SRC in binning.hip) FLAGS="$FLAGS ${BINNING_FLAGS--mllvm -amdgpu-sched-strategy=iterative-ilp}";; esac
  FLAGS="$FLAGS $EXTRA_FLAGS"  # e.g. EXTRA_FLAGS="-mllvm -amdgpu-sched-strategy=iterative-ilp"
  /opt/rocm/bin/hipcc $FLAGS -c $PKG/csrc/.variant_$SRC -o $OUT/${SRC}.o
  rm -f $PKG/csrc/.variant_$SRC
done
OBJS=""
for o in $PKG/build/obj/*.hip.o; do
  b=$(basename $o .o)
  if [ -f $OUT/$b.o ] && [[ " $* " == *" $b "* ]]; then OBJS="$OBJS $OUT/$b.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o $OUT/libgs4d.so
echo "built $OUT/libgs4d.so ($* from $REV)"
