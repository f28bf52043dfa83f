#!/bin/bash
# A/B of the fp32 heads GEMM shapes (GS4D_MLP_SHAPE: 0 kept, 1 dx one row block per wave, 2 dw 64-row m blocks)
set -o pipefail
O=gpurun_out/r06_gemm_ab
mkdir -p $O
for v in 0 1 0; do
  GS4D_MLP_SHAPE=$v timeout -k 10 120 python -u tools/probes/mlp_f32_time.py > $O/time_$v.log 2>&1 || { echo "probe $v failed"; tail -5 $O/time_$v.log; exit 1; }
  echo "shape $v"; cat $O/time_$v.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_gpu.py -k "mlp or heads or train_step" > $O/tests.log 2>&1; tail -2 $O/tests.log
