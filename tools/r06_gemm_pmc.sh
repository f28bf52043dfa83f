#!/bin/bash
# PMC passes over the fp32 heads-block GEMM kernels (one counter group per run); GS4D_MLP_SHAPE passes through
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_pmc_gemm
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/p1 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p1.log 2>&1 || { echo p1 failed; tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE -d $O/p2 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p2.log 2>&1 || { echo p2 failed; tail $O/p2.log; exit 1; }
echo done
