#!/bin/bash
# Kernel traces of the metric-size train step, fp32 and bf16 MLP (tools/probes/train_trace_bf16.py).
export TMPDIR=/tmp
OUT=gpurun_out/trainprof_${TAG:-a}
mkdir -p $OUT
for dt in ${DTYPES:-fp32 bf16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$dt -o run --output-format csv -- python3 tools/probes/train_trace_bf16.py $dt 20 > $OUT/$dt.log 2>&1 || { echo "$dt rc=$?"; tail -5 $OUT/$dt.log; exit 1; }
  grep ms/step $OUT/$dt.log
done
