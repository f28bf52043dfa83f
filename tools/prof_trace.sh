#!/bin/bash
# GPU tests, then a rocprofv3 kernel trace of a short bench into gpurun_out/prof_<tag>.
TAG=${1:-tmp}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/log.txt 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/log.txt; exit 1; }
grep '^{' $OUT/log.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'])"
