#!/bin/bash
# The MLP GEMMs on rocBLAS (TunableOp kernels) vs torch's hipBLASLt picks: GEMM parity + train-step tests,
# then the train-step probe interleaved (GS4D_MLP_ROCBLAS=1 / 0) and one kernel-sequence trace.
export TMPDIR=/tmp
OUT=gpurun_out/ab_mlp_${TAG:-a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in 1 0; do
GS4D_MLP_ROCBLAS=$v timeout -k 10 200 python3 tools/probes/train_trace.py > $OUT/t_${v}_$rep.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/t_${v}_$rep.txt; exit 1; }
echo "rocblas=$v $(grep ms/step $OUT/t_${v}_$rep.txt)"
done; done
TAG=${TAG:-a}_mlp bash tools/train_seq.sh | tail -3
