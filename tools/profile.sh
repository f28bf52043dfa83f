#!/bin/bash
# rocprofv3 evidence for bench.py (MI355X_MICROARCH.md, rocprofv3 sections): a kernel-trace/stats run,
# then FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), then SQ instruction counters -- every
# counter pass with no other trace domain.  Output: gpurun_out/prof_<tag>/{trace,fetch,write,sq}.
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---steps 10 --warmup 3 --no-cpu-baseline --no-train-step}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name, rocprofv3 args...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_$name.log 2>&1 \
        || { echo "$name rc=$?"; tail -20 $OUT/bench_$name.log; exit 1; }
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
find $OUT -name "*.csv" | head -20
