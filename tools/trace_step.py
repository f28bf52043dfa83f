"""Print one step's kernel timeline from a rocprofv3 kernel trace: tools/trace_step.py <run_kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "preprocess_kernel" in n][-3]
t0 = int(rows[idx]["Start_Timestamp"])
end = [i for i, n in enumerate(names) if "preprocess_kernel" in n and i > idx][0]
for r in rows[idx - 2:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:48]:48s} grid={r['Grid_Size_X']} "
          f"vgpr={r['VGPR_Count']} lds={r['LDS_Block_Size']}")
