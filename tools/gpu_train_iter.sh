#!/bin/bash
# Train-step iteration: the train-step kernels' GPU tests, the train-step probe twice, one kernel-sequence trace.
export TMPDIR=/tmp
OUT=gpurun_out/train_iter_${TAG:-a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_train_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
timeout -k 10 200 python3 tools/probes/train_trace.py > $OUT/t_$rep.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/t_$rep.txt; exit 1; }
grep ms/step $OUT/t_$rep.txt
done
TAG=${TAG:-a}_ti bash tools/train_seq.sh | awk '$2>15 || /span/' | cut -c1-110
