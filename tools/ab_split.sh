#!/bin/bash
# A/B of the render backward's two-wave split threshold (GS4D_BWD_SPLIT): parity tests once, then the bench
# (metric + train-like scene stage times) per threshold, interleaved twice.
export TMPDIR=/tmp
OUT=gpurun_out/ab_split_${TAG:-a}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
for thr in ${THRS:-256 0 2000}; do
GS4D_BWD_SPLIT=$thr timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step > $OUT/b_${thr}_$rep.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/b_${thr}_$rep.log; exit 1; }
python - $OUT/b_${thr}_$rep.log $thr <<'PY'
import json,sys
j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
tl=j.get('train_like_scene',{})
print('thr',sys.argv[2],'ms',j['ms_per_step'],'bwd',round(j['stage_ms']['bwd.render_backward']*1e3,1),'fwd',round(j['stage_ms']['fwd.render']*1e3,1),
      '| train_like ms',tl.get('ms_per_step'),'bwd',round(tl.get('stage_ms',{}).get('bwd.render_backward',0)*1e3,1))
PY
done
done
