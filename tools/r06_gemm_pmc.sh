#!/bin/bash
# PMC passes over the fp32 heads-block GEMM kernels (one counter group per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_pmc
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/tools/probes/mlp_f32_run.py 5 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p1 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p1.log 2>&1 || { echo p1 failed; tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE -d $O/p2 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p2.log 2>&1 || { echo p2 failed; tail $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/p3 -o run -- python3 $R/tools/probes/mlp_f32_run.py 3 > $O/p3.log 2>&1 || { echo p3 failed; tail $O/p3.log; exit 1; }
find $O -name "*.csv" | head -20
