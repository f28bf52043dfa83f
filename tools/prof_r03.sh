#!/bin/bash
# Round-3 profiling session: counter list, kernel traces of the metric and train-like scenes, and the
# SQ/TCC counter passes of the metric scene (each --pmc pass alone, no trace domains).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r03a}
mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "list rc=$?"
run() {  # name, rocprofv3 args...; bench args from $BARGS
    local name=$1; shift
    timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS $BARGS > $OUT/bench_$name.log 2>&1 \
        || { echo "$name rc=$?"; tail -20 $OUT/bench_$name.log; exit 1; }
}
BARGS="" run trace --kernel-trace --stats
BARGS="--scene train_like" run trace_tl --kernel-trace --stats
BARGS="" run fetch --pmc FETCH_SIZE
BARGS="" run write --pmc WRITE_SIZE
BARGS="" run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
BARGS="" run sq2 --pmc SQ_INST_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F32 SQ_BUSY_CU_CYCLES
echo done
