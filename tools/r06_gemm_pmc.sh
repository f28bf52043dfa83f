#!/bin/bash
# PMC passes over the fp32 heads-block GEMM kernels (one counter group per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_pmc2
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE -d $O/p2 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p2.log 2>&1 || { echo p2 failed; tail $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p4 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p4.log 2>&1 || { echo p4 failed; tail $O/p4.log; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACCUM_PREV_HIRES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT -d $O/p5 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p5.log 2>&1 || { echo p5 failed; tail $O/p5.log; }
echo done
