#!/bin/bash
# Round-5 evidence on the final tree: the whole GPU suite, smoke(), and the default bench line.
export TMPDIR=/tmp
OUT=gpurun_out/ev_${TAG:-r05}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python3 -c "
import json; j=json.load(open('$OUT/bench.json'))
t=j.get('train_step',{})
print('value', j['value'], 'ms', j['ms_per_step'], 'train', t.get('ms'), 'bf16', t.get('bf16_mlp',{}).get('ms'), 'cpu', j.get('cpu_baseline'))
"
