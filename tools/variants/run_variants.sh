#!/bin/bash
# On the GPU box: time each variants/<name>/libgs4d.so with bench.py's stage timings.
# Usage: tools/variants/run_variants.sh A B C ...   (bench args from $BENCH_ARGS)
LIB=4dgaussians-fast-train_amd/diff_gaussian_rasterization/libgs4d.so
cp $LIB /tmp/libgs4d_intree.so
mkdir -p gpurun_out
for v in "$@"; do
    cp variants/$v/libgs4d.so $LIB
    timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step ${BENCH_ARGS} > gpurun_out/var_$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/var_$v.log; cp /tmp/libgs4d_intree.so $LIB; exit $rc; fi
    grep '^{' gpurun_out/var_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})"
done
cp /tmp/libgs4d_intree.so $LIB
