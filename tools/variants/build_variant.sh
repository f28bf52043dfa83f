#!/bin/bash
# Build a libgs4d.so variant with one translation unit replaced:
#   tools/variants/build_variant.sh <name> <unit, e.g. render> <source path> [extra hipcc flags...]
# Output: variants/<name>/libgs4d.so (the other objects from the last in-tree build).  Diagnostic only.
set -e
NAME=$1; UNIT=$2; SRC=$3; shift 3
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=$ROOT/4dgaussians-fast-train_amd/build/obj
OUT=$ROOT/variants/$NAME
mkdir -p $OUT
NC=""
case $UNIT in render|capi) ;; *) NC="-ffp-contract=off" ;; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-result $NC \
    -I$ROOT/include -I$ROOT/4dgaussians-fast-train_amd/csrc "$@" -c $SRC -o $OUT/$UNIT.o
objs=""
for f in preprocess binning render preprocess_backward knn train_tail hexplane capi; do
    if [ $f = $UNIT ]; then objs="$objs $OUT/$UNIT.o"; else objs="$objs $OBJ/$f.hip.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -o $OUT/libgs4d.so
rm $OUT/$UNIT.o
echo built $OUT/libgs4d.so
