#!/bin/bash
# One GPU session for several A/Bs: the train-step kernel A/B (train_tail variants and knobs), the
# rasterizer A/B (binning variant), then the train-step and parity GPU tests.
export TMPDIR=/tmp
TAG=${TAG:-c} KERNELS="heads_block|feature_bwd|heads_bwd|adam|l1_" bash tools/ab_train_kernels.sh "GS4D_HBF_WG=256" "GS4D_HBF_WG=512" "GS4D_HBF_WG=1024" || exit $?
NO_TESTS=1 TAG=${TAG:-c} VARIANTS="base_bin" bash tools/ab_lib.sh || exit $?
mkdir -p gpurun_out/combo_${TAG:-c}
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/combo_${TAG:-c}/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/combo_${TAG:-c}/tests.log; exit $rc
