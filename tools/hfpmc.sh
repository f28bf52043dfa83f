#!/bin/bash
# PMC passes over the fp32 heads block forward (tools/probes/heads_time.py --fwd32): HBM bytes, MFMA busy,
# LDS and wait counters, one pass per counter group (diagnostic)
export TMPDIR=/tmp
OUT=gpurun_out/prof_hf_${TAG:-a}
mkdir -p $OUT
P="python3 tools/probes/heads_time.py --fwd32"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- $P > $OUT/f.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- $P > $OUT/w.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU -d $OUT/a -o run --output-format csv -- $P > $OUT/a.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES -d $OUT/b -o run --output-format csv -- $P > $OUT/b.txt 2>&1
rc=$?; echo rc=$rc
for d in f w a b; do python3 tools/pmc_kernels.py $OUT/$d heads_block_fwd; done
grep "us" $OUT/f.txt | tail -1
exit $rc
