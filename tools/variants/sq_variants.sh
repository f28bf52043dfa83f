#!/bin/bash
# On the GPU box: one SQ counter pass per variants/<name>/libgs4d.so (plus the in-tree build as "tree"),
# averaged per kernel matching $PAT (default render_).  Usage: tools/variants/sq_variants.sh A B ...
export TMPDIR=/tmp
PAT=${PAT:-render_}
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
cp $LIB /tmp/libgs4d_intree.so
mkdir -p gpurun_out
for v in tree "$@"; do
    [ $v = tree ] || cp variants/$v/libgs4d.so $LIB
    OUT=gpurun_out/sq_$v
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS -d $OUT -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > $OUT.log 2>&1
    rc=$?
    cp /tmp/libgs4d_intree.so $LIB
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 $OUT.log; exit $rc; fi
    echo "== $v"; python3 tools/pmc_kernels.py $OUT $PAT
done
