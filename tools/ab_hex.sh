#!/bin/bash
# hexplane_backward alone per libgs4d variant (tools/build_variant.sh):  VARIANTS="a b" bash tools/ab_hex.sh
export TMPDIR=/tmp
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  echo "== $v"
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 python tools/probes/hex_bwd_time.py || exit 1
done
