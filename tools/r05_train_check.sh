#!/bin/bash
# Train-step check on one box: the train GPU tests (+ the short convergence comparison), the fp32 / bf16
# train-step kernel sequences, and a bench line without the CPU baseline.  Stops at the first failure.
export TMPDIR=/tmp
OUT=gpurun_out/tc_${TAG:-r05}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_training_quality_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread -k "${TESTS_K:-not long_horizon}" > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" $OUT/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
TAG=${TAG}_f32 bash tools/train_seq.sh | tail -1 || exit 1
PROBE_ARGS="metric --bf16" TAG=${TAG}_bf16 bash tools/train_seq.sh | tail -1 || exit 1
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); t=j.get('train_step',{})
print('value', j['value'], 'ms', j['ms_per_step'], 'train', t.get('ms'), 'bf16', (t.get('bf16_mlp') or {}).get('ms'))
"
