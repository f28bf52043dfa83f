#!/bin/bash
# Round-3 final evidence on one box: the whole GPU suite, smoke(), the default bench line, then the profile passes
# (kernel trace + PMC of the metric scene, kernel trace of the train-like scene, the train step's kernel split).
export TMPDIR=/tmp
TAG=${TAG:-r03f} bash tools/r03_evidence.sh || exit $?
TAG=${TAG:-r03f} bash tools/prof_valu.sh || exit $?
OUT=gpurun_out/prof_${TAG:-r03f}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_tl -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras --scene train_like > $OUT/bench_trace_tl.log 2>&1 || { echo "trace_tl rc=$?"; exit 1; }
TAG=${TAG:-r03f} bash tools/train_seq.sh | tail -1
echo final done
