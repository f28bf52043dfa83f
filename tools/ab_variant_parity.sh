#!/bin/bash
# Parity tests of a libgs4d variant (VARIANT=<name>), then the bench A/B of the current build against it.
export TMPDIR=/tmp
OUT=gpurun_out/ab_var_${TAG:-a}
mkdir -p $OUT
LD_LIBRARY_PATH=4dgaussians-fast-train_amd/build/variant_$VARIANT${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "variant pytest rc=$rc"; grep -o "'flagged_pix': [0-9]*" $OUT/tests.log | sort | uniq -c | sort -rn | head -3; tail -2 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
NO_TESTS=1 TAG=${TAG:-a} VARIANTS="$VARIANT" bash tools/ab_lib.sh
