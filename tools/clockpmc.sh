#!/bin/bash
# Effective clock of each kernel of a probe (diagnostic): GRBM_GUI_ACTIVE / 8 XCDs / kernel duration,
# counters and kernel trace in one run (no other trace domain).   tools/clockpmc.sh <probe args...>
export TMPDIR=/tmp
OUT=gpurun_out/clock_${TAG:-a}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $OUT/p -o run --output-format csv -- python3 "$@" > $OUT/log.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/log.txt; exit 1; }
python3 - $OUT/p <<'PY'
import csv, glob, sys
from collections import defaultdict
src = sys.argv[1]
cnt = {}
for f in glob.glob(src + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = r.get("Correlation_Id") or r.get("Dispatch_Id")
        cnt.setdefault(key, {"name": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
dur = {}
for f in glob.glob(src + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = r.get("Correlation_Id") or r.get("Dispatch_Id")
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
agg = defaultdict(list)
for k, v in cnt.items():
    if k in dur and "GRBM_GUI_ACTIVE" in v and dur[k] > 0:
        agg[v["name"].split("(")[0][:70]].append((v["GRBM_GUI_ACTIVE"] / 8 / dur[k], dur[k] / 1e3))
for n, xs in sorted(agg.items(), key=lambda t: -sum(x[1] for x in t[1])):
    xs.sort()
    print(f"{n:72s} n={len(xs):3d} clock {xs[len(xs)//2][0]:.2f} GHz  dur {sorted(x[1] for x in xs)[len(xs)//2]:8.1f} us")
PY
