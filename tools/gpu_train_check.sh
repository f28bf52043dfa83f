#!/bin/bash
# On the GPU box: train-step GPU tests, then the train-step timing probe (and its kernel trace with TRACE=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/probes/train_trace.py > gpurun_out/train_time.txt 2>&1 || exit $?
grep train_step gpurun_out/train_time.txt
if [ -n "$TRACE" ]; then
  mkdir -p gpurun_out/prof_train && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train/trace -o run --output-format csv -- python3 tools/probes/train_trace.py > gpurun_out/prof_train/log.txt 2>&1 || exit $?
  python3 tools/kstats.py gpurun_out/prof_train/trace 25 30
fi
