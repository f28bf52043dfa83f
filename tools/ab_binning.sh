mkdir -p gpurun_out; export TMPDIR=/tmp
for m in radix count radix count; do
  if [ $m = radix ]; then export GS4D_BINNING=radix; else unset GS4D_BINNING; fi
  echo "== $m"; timeout -k 10 200 python tools/train_step_bench.py --modes fused+hex --steps 60 --warmup 10 || exit $?
done
