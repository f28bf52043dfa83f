#!/bin/bash
# One iteration on the GPU box: rasterizer parity tests, a short bench, kernel traces of the metric and
# train-like scenes.  Stops at the first failing step (nothing more touches the GPU after a fault).
export TMPDIR=/tmp
OUT=gpurun_out/iter_${TAG:-x}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q -s --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:---no-train-step} > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json,sys
j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('value',j['value'],'ms',j['ms_per_step'],'L',j['num_rendered'])
print({k:v for k,v in j['stage_ms'].items()})
for k in ('autograd_wrapper','train_like_scene','train_step'):
    if k in j: print(k, j[k] if k!='train_like_scene' else {kk:j[k][kk] for kk in ('ms_per_step','stage_ms')})
PY
[ -n "$NO_TRACE" ] && exit 0
for sc in synthetic train_like; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/tr_$sc -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras --scene $sc > $OUT/tr_$sc.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python - $OUT/tr_$sc/run_kernel_stats.csv $sc <<'PY'
import csv,sys
print(sys.argv[2], ' '.join('%s=%.1f'%(r['Name'].split('(')[0].replace('gs4d::','').replace('void ','')[:28], float(r['AverageNs'])/1e3) for r in list(csv.DictReader(open(sys.argv[1])))[:14]))
PY
done
