#!/bin/bash
# Train-step wall time with torch's GEMM selection as is, then with TunableOp tuning the hipBLASLt/rocBLAS
# solution of every GEMM shape on first use (results written to gpurun_out/tunableop/), then re-using them.
export TMPDIR=/tmp
OUT=gpurun_out/tunableop
mkdir -p $OUT
timeout -k 10 200 python3 tools/probes/train_trace.py > $OUT/plain.txt 2>&1 || { echo "plain rc=$?"; tail -5 $OUT/plain.txt; exit 1; }
grep ms/step $OUT/plain.txt
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/results%d.csv \
  timeout -k 10 400 python3 tools/probes/train_trace.py > $OUT/tune.txt 2>&1 || { echo "tune rc=$?"; tail -5 $OUT/tune.txt; exit 1; }
grep ms/step $OUT/tune.txt
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/results%d.csv \
  timeout -k 10 200 python3 tools/probes/train_trace.py > $OUT/tuned.txt 2>&1 || { echo "tuned rc=$?"; tail -5 $OUT/tuned.txt; exit 1; }
grep ms/step $OUT/tuned.txt
cat $OUT/results0.csv 2>/dev/null | cut -c1-200
