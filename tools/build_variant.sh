#!/bin/bash
# Build libgs4d with ONE source file taken from a git revision (default HEAD) into
# 4dgaussians-fast-train_amd/build/variant_<name>/libgs4d.so, every other object from the current build:
#   tools/build_variant.sh <name> <csrc file> [rev]
# A/B on the box: LD_LIBRARY_PATH=4dgaussians-fast-train_amd/build/variant_<name> python bench.py ...
# (the bindings' RUNPATH yields to LD_LIBRARY_PATH).
set -e
NAME=$1; SRC=$2; REV=${3:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/4dgaussians-fast-train_amd
OUT=$PKG/build/variant_$NAME
mkdir -p $OUT
git -C $ROOT show $REV:4dgaussians-fast-train_amd/csrc/$SRC > $PKG/csrc/.variant_$SRC
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-result -I$ROOT/include"
case $SRC in preprocess.hip|binning.hip|preprocess_backward.hip|knn.hip|train_tail.hip|hexplane.hip) FLAGS="$FLAGS -ffp-contract=off";; esac
/opt/rocm/bin/hipcc $FLAGS -c $PKG/csrc/.variant_$SRC -o $OUT/${SRC}.o
rm -f $PKG/csrc/.variant_$SRC
OBJS=""
for o in $PKG/build/obj/*.hip.o; do
  if [ "$(basename $o)" = "$SRC.o" ]; then OBJS="$OBJS $OUT/${SRC}.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o $OUT/libgs4d.so
echo "built $OUT/libgs4d.so ($SRC from $REV)"
