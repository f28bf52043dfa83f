"""Per-kernel averages from rocprofv3 SQLite outputs (run_results.db): kernel durations and PMC counter values.
Usage: python tools/pmc_db.py <db> [<db> ...] [--match SUBSTR]"""
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match in args:
    args.remove(match)
for db in args:
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")} \
        if "kernel_name" in [r[1] for r in c.execute("pragma table_info(rocpd_info_kernel_symbol)")] else \
        {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    dur = defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        dur[kid].append((e - s) / 1e3)
    pmc = defaultdict(lambda: defaultdict(list))
    pmcname = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    q = ("select d.kernel_id, p.pmc_id, p.value from rocpd_pmc_event p join rocpd_kernel_dispatch d "
         "on p.event_id = d.event_id")
    try:
        for kid, pid, v in c.execute(q):
            pmc[kid][pmcname.get(pid, pid)].append(v)
    except sqlite3.Error as e:
        print("pmc join failed:", e)
    print(f"== {db}")
    for kid, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        n = names.get(kid, str(kid))
        if match and match not in n:
            continue
        line = f"{n[:70]:70s} n={len(ds):3d} avg {sum(ds) / len(ds):9.1f} us"
        for k, vs in sorted(pmc[kid].items()):
            per = sum(vs) / len(ds)
            line += f" | {k}={per:.4g}"
        print(line)
