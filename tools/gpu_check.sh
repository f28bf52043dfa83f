#!/bin/bash
# One GPU session: parity tests, then (only if nothing crashed) a short bench.
# Exit statuses >= 124 (timeout/abort/segfault) stop the session: nothing more touches the GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q -s ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -3 gpurun_out/bench.log
exit $brc
