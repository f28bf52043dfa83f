#!/bin/bash
# A/B of the deformation heads' kernels across libgs4d variants (tools/build_variant.sh): heads_time.py per
# library.   VARIANTS="a b" bash tools/ab_heads.sh
OUT=gpurun_out/ab_heads_${TAG:-a}
mkdir -p $OUT
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 python tools/probes/heads_time.py > $OUT/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep " us" $OUT/$v.log
done
