#!/bin/bash
# A/B of libgs4d variants (tools/build_variant.sh) on a timing probe: PROBE (default
# tools/probes/small_kernels_time.py) once per library, twice.   VARIANTS="a b" PROBE=... bash tools/ab_probe.sh
OUT=gpurun_out/ab_probe_${TAG:-a}
mkdir -p $OUT
for rep in 1 2; do
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 python ${PROBE:-tools/probes/small_kernels_time.py} > $OUT/${v}_$rep.log 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/${v}_$rep.log; exit 1; }
  echo "== $v"; grep " us" $OUT/${v}_$rep.log
done; done
