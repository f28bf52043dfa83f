#!/bin/bash
# On the GPU box: one rocprofv3 --pmc pass per variants/<name>/libgs4d.so over a short bench run.
# Usage: COUNTERS="SQ_..." tools/variants/pmc_variants.sh A B ...  -> gpurun_out/pmcv_<name>/
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
export TMPDIR=/tmp
CNT=${COUNTERS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU}
cp $LIB /tmp/libgs4d_intree.so
for v in "$@"; do
    cp variants/$v/libgs4d.so $LIB
    mkdir -p gpurun_out/pmcv_$v
    timeout -s KILL 120 rocprofv3 --pmc $CNT -d gpurun_out/pmcv_$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train-step > gpurun_out/pmcv_$v/log.txt 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/pmcv_$v/log.txt; cp /tmp/libgs4d_intree.so $LIB; exit 1; fi
    python3 tools/pmc_kernels.py gpurun_out/pmcv_$v render
done
cp /tmp/libgs4d_intree.so $LIB
