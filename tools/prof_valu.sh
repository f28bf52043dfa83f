#!/bin/bash
# Measured VALU utilisation of the blend kernels (the counters VERDICT r02 asked for): rocprof's derived
# VALUBusy / VALUUtilization plus the raw SQ counters they come from, each pass alone (no trace domains).
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-valu}
mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras"
run() {
    local name=$1; shift
    timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_$name.log 2>&1 \
        || { echo "$name rc=$?"; tail -20 $OUT/bench_$name.log; exit 1; }
}
run trace --kernel-trace --stats
run derived --pmc VALUBusy VALUUtilization
run grbm --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo done
