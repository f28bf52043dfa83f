# Tail/occupancy probe: the blend kernels launched with every tile repeated GS4D_DUP times (temporary
# build; idempotent writes), kernel time vs repeat count.
export TMPDIR=/tmp
mkdir -p gpurun_out/dup
for d in 1 2 3; do
  GS4D_DUP=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dup/d$d -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-train-step --no-extras ${SCENE:+--scene $SCENE} > gpurun_out/dup/d$d.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/dup/d$d/run_kernel_stats.csv')):
    if 'render_' in r['Name']: print('dup $d', r['Name'][:30], round(float(r['AverageNs'])/1e3,1))"
done
