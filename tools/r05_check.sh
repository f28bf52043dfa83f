#!/bin/bash
# Round-5 check on one box: the rasterizer parity suite (with the flip-band measurement), the train-step GPU
# tests, kernel traces of the metric and train-like scenes, the fp32 / bf16 train-step kernel sequences, and a
# bench line without the CPU baseline.  Each GPU step has its own time limit; the script stops at the first
# failure.
export TMPDIR=/tmp
OUT=gpurun_out/c_${TAG:-r05}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_train_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread -s > $OUT/tests.log 2>&1
rc=$?; grep -E "pairs within|passed|failed|Error" $OUT/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_m -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace_m.log 2>&1 || { echo "trace_m rc=$?"; exit 1; }
python3 tools/kstats.py $OUT/trace_m 13 8
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_tl -o run --output-format csv -- python3 bench.py $ARGS --scene train_like > $OUT/trace_tl.log 2>&1 || { echo "trace_tl rc=$?"; exit 1; }
python3 tools/kstats.py $OUT/trace_tl 13 8
TAG=${TAG}_f32 bash tools/train_seq.sh | tail -1 || exit 1
PROBE_ARGS="metric --bf16" TAG=${TAG}_bf16 bash tools/train_seq.sh | tail -1 || exit 1
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); t=j.get('train_step',{})
print('value', j['value'], 'ms', j['ms_per_step'], 'train fp32', t.get('ms'), 'bf16', t.get('bf16_mlp',{}).get('ms'))
"
