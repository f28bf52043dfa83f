"""Print the top kernels of a rocprofv3 kernel_stats.csv: python tools/kstats.py <csv or dir> [steps] [top]."""
import csv
import glob
import os
import sys


def main():
    src = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    if os.path.isdir(src):
        src = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(src)))
    tot = sum(float(x["TotalDurationNs"]) for x in rows)
    print(f"total {tot / 1e6 / steps:.3f} ms per step ({steps:g} steps)")
    for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:top]:
        print(f"{x['Name'][:66]:66s} {x['Calls']:>6s} {float(x['AverageNs']) / 1000:9.2f}us "
              f"{float(x['TotalDurationNs']) / 1e6 / steps:8.3f}ms/step")


if __name__ == "__main__":
    main()
