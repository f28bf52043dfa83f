#!/bin/bash
# On the GPU box: kernel trace (rocprofv3 --kernel-trace --stats) of bench.py with each
# variants/<name>/libgs4d.so in turn; prints the top kernels.  Usage: tools/variants/trace_variants.sh A B ..
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
cp $LIB /tmp/libgs4d_intree.so
for v in "$@"; do
    if [ "$v" = intree ]; then cp /tmp/libgs4d_intree.so $LIB; else cp variants/$v/libgs4d.so $LIB; fi
    echo "== $v"
    bash tools/trace_only.sh var_$v --steps 10 --warmup 3 --no-cpu-baseline --no-train-step | head -14 || { cp /tmp/libgs4d_intree.so $LIB; exit 1; }
done
cp /tmp/libgs4d_intree.so $LIB
