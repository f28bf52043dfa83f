#!/bin/bash
# Build a libgs4d.so variant: tools/variants/build_variant.sh <name> <render.hip source> [extra hipcc flags...]
# Output: variants/<name>/libgs4d.so (other objects from the last in-tree build).  Diagnostic only.
set -e
NAME=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=$ROOT/4dgaussians-fast-train_amd/build/obj
OUT=$ROOT/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-result \
    -I$ROOT/include -I$ROOT/4dgaussians-fast-train_amd/csrc "$@" -c $SRC -o $OUT/render.o
objs=""
for f in preprocess binning preprocess_backward knn train_tail hexplane capi; do objs="$objs $OBJ/$f.hip.o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $OUT/render.o -o $OUT/libgs4d.so
rm $OUT/render.o
echo built $OUT/libgs4d.so
