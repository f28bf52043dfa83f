export TMPDIR=/tmp
OUT=gpurun_out/prof_hex
mkdir -p $OUT
cd tools/probes
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d ../../$OUT/a -o run --output-format csv -- python3 hexplane_probe.py > ../../$OUT/a.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU -d ../../$OUT/b -o run --output-format csv -- python3 hexplane_probe.py > ../../$OUT/b.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_ATOMIC_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum SQ_INSTS_VMEM_WR -d ../../$OUT/c -o run --output-format csv -- python3 hexplane_probe.py > ../../$OUT/c.txt 2>&1
echo rc=$?
