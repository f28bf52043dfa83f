#!/bin/bash
# Kernel-trace summary of a short bench run: gpurun_out/prof_$1/ (per-kernel average µs printed).
TAG=${1:-q}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-step > $OUT/log.txt 2>&1 || { echo "rc=$?"; tail -20 $OUT/log.txt; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs'])):
    print(f"{x['Name'][:58]:58s} {x['Calls']:>5s} {float(x['AverageNs'])/1000:8.2f}us")
PY
grep '^{' $OUT/log.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})"
