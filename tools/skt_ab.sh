#!/bin/bash
# Kernel-trace A/B of libgs4d variants (tools/build_variant.sh) on tools/probes/small_kernels_time.py:
# VARIANTS="a b" bash tools/skt_ab.sh -- per-kernel average durations for the current build and each variant.
export TMPDIR=/tmp
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  mkdir -p gpurun_out/skt_ab/$v
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/skt_ab/$v -o run --output-format csv -- python3 tools/probes/small_kernels_time.py > gpurun_out/skt_ab/$v/log.txt 2>&1 || { echo "$v rc=$?"; exit 1; }
  echo "== $v"; python3 tools/kstats.py gpurun_out/skt_ab/$v 13 6 | grep -E "reg_backward|l1_partial|feature"
done
