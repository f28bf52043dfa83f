#!/bin/bash
# A/B of libgs4d variants (tools/build_variant.sh) against the current build on one box: parity tests on the
# current build, then the bench (metric + train-like stage times) per library, interleaved twice.
#   VARIANTS="base other" bash tools/ab_lib.sh
export TMPDIR=/tmp
OUT=gpurun_out/ab_lib_${TAG:-a}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-train-step > $OUT/b_${v}_$rep.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/b_${v}_$rep.log; exit 1; }
  python - $OUT/b_${v}_$rep.log $v <<'PY'
import json,sys
j=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
tl=j.get('train_like_scene',{}); st=tl.get('stage_ms',{})
km=j.get('kernel_ms',{})
print(f"{sys.argv[2]:8s} ms {j['ms_per_step']} fwd {j['stage_ms']['fwd.render']*1e3:.1f} bwd {j['stage_ms']['bwd.render_backward']*1e3:.1f} (kernel {km.get('fwd.render',0)*1e3:.1f} / {km.get('bwd.render_backward',0)*1e3:.1f}) bin {j['stage_ms']['fwd.binning']*1e3:.1f} | train_like ms {tl.get('ms_per_step')} fwd {st.get('fwd.render',0)*1e3:.1f} bwd {st.get('bwd.render_backward',0)*1e3:.1f} bin {st.get('fwd.binning',0)*1e3:.1f}")
PY
done
done
