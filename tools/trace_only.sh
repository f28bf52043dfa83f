#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py only (quick look at the kernel split).
# Usage: tools/trace_only.sh <tag> [bench args...]
TAG=${1:-q}; shift
ARGS=${@:---steps 20 --warmup 5 --no-cpu-baseline --no-train-step}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || exit $?
python3 tools/kstats.py $OUT/trace 25 30
