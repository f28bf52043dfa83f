#!/bin/bash
# round 6: the f32-MFMA heads GEMMs (timing, parity, cross-process bits), HexPlane bound + race fix, row surgery,
# and the short-horizon training spread
set -o pipefail
O=gpurun_out/r06_gemm
mkdir -p $O
timeout -k 10 180 python -u tools/probes/mlp_f32_time.py > $O/time.log 2>&1 || { echo "probe failed"; tail -20 $O/time.log; exit 1; }
cat $O/time.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -5 $O/tests.log
timeout -k 10 180 python -u tools/probes/hex_heavy_tail.py > $O/heavy.log 2>&1 || { echo "heavy failed"; tail -20 $O/heavy.log; exit 1; }
cat $O/heavy.log
timeout -k 10 300 python -u tools/probes/conv_spread.py 12 0 > $O/spread_a.log 2>&1 || { echo "spread a failed"; tail -20 $O/spread_a.log; exit 1; }
timeout -k 10 300 python -u tools/probes/conv_spread.py 12 0 > $O/spread_b.log 2>&1 || { echo "spread b failed"; tail -20 $O/spread_b.log; exit 1; }
tail -3 $O/spread_a.log $O/spread_b.log
