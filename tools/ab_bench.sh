#!/bin/bash
# A/B of environment knobs on bench.py in one box: tools/ab_bench.sh "ENV=a" "ENV=b" ...  ("-" = no env)
export TMPDIR=/tmp
for round in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then e=""; else e="$cfg"; fi
    echo "== $cfg"
    env $e timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-train-step 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stage_ms'])" || exit $?
  done
done
