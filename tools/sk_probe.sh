#!/bin/bash
# Kernel trace of the split-K chunk probe, one run per chunk size (tools/probes/splitk_chunk.py): the kernels of
# the 10 steady calls after the probe's marker fill, averaged per call.
export TMPDIR=/tmp
for c in "$@"; do
  mkdir -p gpurun_out/sk/$c
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/sk/$c -o run --output-format csv -- python3 tools/probes/splitk_chunk.py $c > gpurun_out/sk/$c/log.txt 2>&1 || exit 1
  echo "== $c"; grep kChunk gpurun_out/sk/$c/log.txt
  python3 - gpurun_out/sk/$c <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
m = max(i for i, r in enumerate(rows) if "FillFunctor" in r["Kernel_Name"])
tot = defaultdict(float)
for r in rows[m + 1:]:
    tot[r["Kernel_Name"][:70]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / 10
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {v:8.1f} us/call  {k}")
print(f"  {sum(tot.values()):8.1f} us/call total")
PY
done
