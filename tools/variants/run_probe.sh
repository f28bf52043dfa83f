#!/bin/bash
# On the GPU box: run a probe script against each variants/<name>/libgs4d.so.
# Usage: tools/variants/run_probe.sh <probe.py> A B ...
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
PROBE=$1; shift
cp $LIB /tmp/libgs4d_intree.so
mkdir -p gpurun_out
for v in "$@"; do
    cp variants/$v/libgs4d.so $LIB
    echo "== variant $v"
    timeout -k 10 120 python $PROBE > gpurun_out/probe_$v.log 2>&1
    rc=$?
    grep -v amdgpu.ids gpurun_out/probe_$v.log
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; cp /tmp/libgs4d_intree.so $LIB; exit $rc; fi
done
cp /tmp/libgs4d_intree.so $LIB
