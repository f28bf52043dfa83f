# PMC passes over tools/probes/heads_bwd_probe.py (diagnostic)
export TMPDIR=/tmp
OUT=gpurun_out/prof_hb
mkdir -p $OUT
cd tools/probes
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d ../../$OUT/a -o run --output-format csv -- python3 heads_bwd_probe.py > ../../$OUT/a.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU -d ../../$OUT/b -o run --output-format csv -- python3 heads_bwd_probe.py > ../../$OUT/b.txt 2>&1
echo rc=$?
