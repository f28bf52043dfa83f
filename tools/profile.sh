#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md §rocprofv3: TCC slots; never combined with other trace domains).
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---steps 20 --warmup 5 --no-cpu-baseline}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $OUT/bench_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1 || { echo "fetch rc=$?"; tail -20 $OUT/bench_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1 || { echo "write rc=$?"; tail -20 $OUT/bench_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
