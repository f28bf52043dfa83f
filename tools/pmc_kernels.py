"""Average PMC counter values per dispatch for kernels whose name contains a pattern:
python tools/pmc_kernels.py <rocprofv3 output dir> <pattern>."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    src, pat = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                name = r["Kernel_Name"].split("(")[0]
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, d in sorted(acc.items()):
        print(name, {k: round(sum(v) / len(v)) for k, v in sorted(d.items())})


if __name__ == "__main__":
    main()
