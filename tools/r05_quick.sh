#!/bin/bash
# Round-5 quick look on one box: the flip-band measurement and parity tests named by $TESTS_K, kernel traces
# of the metric and train-like scenes (rocprofv3 --kernel-trace --stats, summarised by tools/kstats.py),
# and a bench line without the CPU baseline.
export TMPDIR=/tmp
OUT=gpurun_out/q_${TAG:-r05}
mkdir -p $OUT
if [ -n "$TESTS_K" ]; then
  timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 400 --timeout-method thread -k "$TESTS_K" > $OUT/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "pairs within|PASS|FAIL|Error|assert" $OUT/tests.log | tail -30
  [ $rc -ne 0 ] && exit $rc
fi
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_m -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace_m.log 2>&1 || { echo "trace_m rc=$?"; tail -5 $OUT/trace_m.log; exit 1; }
python3 tools/kstats.py $OUT/trace_m 13 14
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_tl -o run --output-format csv -- python3 bench.py $ARGS --scene train_like > $OUT/trace_tl.log 2>&1 || { echo "trace_tl rc=$?"; tail -5 $OUT/trace_tl.log; exit 1; }
python3 tools/kstats.py $OUT/trace_tl 13 14
timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | python3 -c "
import json,sys; j=json.loads(sys.stdin.read())
ts=j.get('train_step',{})
print('value', j['value'], 'ms', j['ms_per_step'], 'stage', j.get('stage_ms'), 'train', ts.get('ms_per_step'), 'bf16', ts.get('bf16_mlp',{}).get('ms_per_step') if isinstance(ts.get('bf16_mlp'),dict) else ts.get('bf16_mlp'))
"
