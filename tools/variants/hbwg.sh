# fused heads forward: workgroups per launch (temporary env knob GS4D_HBF_WG)
export TMPDIR=/tmp
for wg in 256 512 1024; do
  GS4D_HBF_WG=$wg DTYPES=fp32 TAG=hbwg$wg bash tools/train_prof.sh || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/trainprof_hbwg$wg/fp32/run_kernel_stats.csv')):
    if 'heads_block' in r['Name']: print('wg $wg', round(float(r['AverageNs'])/1e3,1))"
done
