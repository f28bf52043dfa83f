for rep in 1 2; do
for v in 8 16 4; do
GS4D_COUNT_MIN_ITEMS=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-train-step > gpurun_out/abenv_$v.log 2>&1 || exit 1
python3 - gpurun_out/abenv_$v.log $v <<'PY'
import json,sys
j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
tl=j.get('train_like_scene',{}); st=tl.get('stage_ms',{})
print(sys.argv[2], 'metric bin', round(j['stage_ms']['fwd.binning']*1e3,1), 'ms', j['ms_per_step'], '| train_like bin', round(st.get('fwd.binning',0)*1e3,1), 'ms', tl.get('ms_per_step'))
PY
done; done
