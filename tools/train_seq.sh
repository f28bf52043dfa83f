#!/bin/bash
# One train step's kernel sequence (rocprofv3 kernel trace of tools/probes/train_trace.py), anchored on the
# Adam launch that ends each step: start offset, duration and name of every kernel between two of them.
export TMPDIR=/tmp
OUT=gpurun_out/trainseq_${TAG:-a}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 ${PROBE:-tools/probes/train_trace.py} ${PROBE_ARGS} > $OUT/log.txt 2>&1 || { echo "rc=$?"; tail -20 $OUT/log.txt; exit 1; }
cat $OUT/log.txt | grep ms/step
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY' | tee $OUT/seq.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
ad = [i for i, n in enumerate(names) if "adam_kernel" in n]
a, b = ad[-3], ad[-2]
t0 = int(rows[a]["End_Timestamp"])
busy = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:100]}")
print(f"step span {(int(rows[b]['End_Timestamp']) - t0) / 1000:.1f} us, kernel busy {busy / 1000:.1f} us, {b - a} launches")
PY
