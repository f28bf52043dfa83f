#!/bin/bash
# Round-6 profiles on one box: kernel trace + PMC passes of the metric scene (tools/prof_valu.sh), the kernel
# trace of the train-like scene, the train step's kernel sequence (fp32 and bf16 MLP), the fp32 heads block
# forward's PMC passes and the fp32 heads GEMMs' PMC passes.
export TMPDIR=/tmp
T=${TAG:-r06}
TAG=$T bash tools/prof_valu.sh || exit $?
OUT=gpurun_out/prof_$T
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_tl -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras --scene train_like > $OUT/bench_trace_tl.log 2>&1 || { echo "trace_tl rc=$?"; exit 1; }
TAG=$T bash tools/train_seq.sh | tail -1 || exit 1
PROBE_ARGS="metric --bf16" TAG=${T}_bf16 bash tools/train_seq.sh | tail -1 || exit 1
TAG=$T bash tools/hfpmc.sh | tail -3 || exit 1
bash tools/r06_gemm_pmc.sh || exit 1
echo profiles done
