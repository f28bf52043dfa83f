#!/bin/bash
# round 6: the f32-MFMA heads GEMMs (timing, one PMC pass), the train GPU tests, the training-quality short test.
# A test failure (rc 1) does not stop the later steps; anything else does.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_gemm
mkdir -p $O
timeout -k 10 180 python -u tools/probes/mlp_f32_time.py > $O/time.log 2>&1 || { echo "probe failed"; tail -20 $O/time.log; exit 1; }
grep "P=" $O/time.log
timeout -k 10 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p1 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p1.log 2>&1 || { echo p1 failed; tail $O/p1.log; exit 1; }
timeout -k 10 700 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_train_gpu.py > $O/tests.log 2>&1
rc=$?
tail -4 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_training_quality_gpu.py -k short > $O/short.log 2>&1
tail -3 $O/short.log
