#!/bin/bash
# On the GPU box: rasterizer parity tests on the in-tree build, its bench stage times, then the
# stage times of each variants/<name>/libgs4d.so.  Usage: tools/variants/parity_and_time.sh A B ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step > gpurun_out/var_tree.log 2>&1 || exit $?
grep '^{' gpurun_out/var_tree.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tree', d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})"
[ $# -gt 0 ] && bash tools/variants/run_variants.sh "$@"
exit 0
