#!/bin/bash
# SQ counters of the blend kernels for the current libgs4d and variants (tools/build_variant.sh), one pass
# per counter set and library, each alone (no trace domains):  VARIANTS="base" bash tools/sq_ab.sh
export TMPDIR=/tmp
OUT=gpurun_out/sq_${TAG:-ab}
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-train-step --no-extras ${SCENE:+--scene $SCENE}"
SETS=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE")
for v in cur $VARIANTS; do
  if [ $v = cur ]; then LP=""; else LP="4dgaussians-fast-train_amd/build/variant_$v"; fi
  i=0
  for s in "${SETS[@]}"; do
    LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 rocprofv3 --pmc $s -d $OUT/${v}_$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/${v}_$i.log 2>&1 || { echo "$v $i rc=$?"; tail -5 $OUT/${v}_$i.log; exit 1; }
    echo "== $v set $i"; python3 tools/pmc_kernels.py $OUT/${v}_$i render_
    i=$((i+1))
  done
done
