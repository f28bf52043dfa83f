#!/bin/bash
# Kernel-time A/B of train-step configurations: for each "ENV=.. ENV2=.." config (LIB=<variant> selects
# 4dgaussians-fast-train_amd/build/variant_<variant>/libgs4d.so), a rocprofv3 kernel trace of
# tools/probes/train_trace.py and the average µs of the kernels matching $KERNELS (regex).
#   KERNELS="heads_block|feature_bwd" bash tools/ab_train_kernels.sh "GS4D_HBF_WG=256" "LIB=base" ...
export TMPDIR=/tmp
OUT=gpurun_out/ab_tk_${TAG:-a}
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=""; lp=""
  for kv in $cfg; do
    case $kv in LIB=*) lp="4dgaussians-fast-train_amd/build/variant_${kv#LIB=}";; -) ;; *) envs="$envs $kv";; esac
  done
  env $envs LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/c$i -o run --output-format csv -- python3 tools/probes/train_trace.py > $OUT/c$i.log 2>&1 || { echo "cfg $cfg rc=$?"; tail -5 $OUT/c$i.log; exit 1; }
  f=$(find $OUT/c$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$cfg" "${KERNELS:-.}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if re.search(sys.argv[3], r['Name'])]
tot = sum(float(r['TotalDurationNs']) for r in rows) / 1e3
print(f"[{sys.argv[2]}] total {tot:.0f} us | " + "  ".join(f"{r['Name'].split('(')[0].replace('gs4d::','').replace('void ','')[:26]}={float(r['AverageNs'])/1e3:.1f}" for r in sel))
PY
done
