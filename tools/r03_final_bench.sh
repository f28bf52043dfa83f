#!/bin/bash
# The final tree's default bench line and the train step's kernel sequence (profiles/r03_bench.json,
# r03_train_step_*).
export TMPDIR=/tmp
OUT=gpurun_out/finalbench
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python3 -c "import json; j=json.load(open('$OUT/bench.json')); print('value', j['value'], 'ms', j['ms_per_step'], 'train', j['train_step']['ms'])"
TAG=final bash tools/train_seq.sh | tail -1
