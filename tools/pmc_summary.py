"""Summarise a tools/profile.sh run into profiles/: per-kernel average duration (kernel trace) and HBM
traffic per launch from FETCH_SIZE (doubled: gfx950 tallies 128-B read requests at 64 B,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, and SQ instruction counts.

  python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>_   -> <prefix>kernel_stats.csv,
  <prefix>pmc.json, profiles/pmc_traffic.json (read by bench.py for roofline.traffic) and
  profiles/pmc_valu.json (VALU wave-instructions per launch, for bench.py's issue-bound figure).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

KEYS = {"gaussian_sh_backward_kernel": "gaussian_sh_backward", "render_backward_kernel": "render_backward", "render_forward_kernel": "render",
        "onesweep_kernel": "onesweep", "emit_instances_kernel": "emit_instances", "preprocess_kernel": "preprocess",
        "contrib_segments_kernel": "contrib_segments", "gaussian_backward_kernel": "gaussian_backward",
        "visible_scan_kernel": "visible_scan", "tile_ranges_kernel": "tile_ranges",
        "tile_sort_kernel": "tile_sort", "tile_order_kernel": "tile_order",
        "contrib_finish_kernel": "contrib_finish", "tile_count_kernel": "tile_count",
        "tile_scan_kernel": "tile_scan", "tile_scatter_kernel": "tile_scatter",
        "sh_backward_kernel": "sh_backward"}


def short(name):
    for k, v in KEYS.items():
        if k in name:
            return v
    return None


def counters(path):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, prefix + "kernel_stats.csv")
    res = {}
    per_kernel = defaultdict(dict)
    for part in ("fetch", "write", "sq", "derived", "grbm"):
        if not os.path.isdir(os.path.join(src, part)):
            continue
        c = counters(os.path.join(src, part))
        for k, d in c.items():
            for name, vals in d.items():
                # rocprofv3 reports one row per dispatch (summed over dimensions)
                per_kernel[k][name] = sum(vals) / len(vals)
    traffic, raw = {}, {}
    for k, d in per_kernel.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            # FETCH_SIZE / WRITE_SIZE are in KiB
            traffic[k] = round((2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0)
            raw[k] = round((d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0)
    res["per_kernel"] = per_kernel
    res["hbm_bytes_per_launch"] = traffic
    res["raw_fetch_plus_write_bytes_per_launch"] = raw
    res["note"] = ("hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 per dispatch; the x2 read "
                   "correction is MI355X_MICROARCH.md §HBM's for gfx950 wide coalesced streaming reads (other access "
                   "widths are uncalibrated: the blend kernels' reads are mostly 8-16 B gathers, so their corrected "
                   "figure is an upper bound and raw_fetch_plus_write_bytes_per_launch a lower one); Infinity-Cache "
                   "hits are counted")
    json.dump(res, open(prefix + "pmc.json", "w"), indent=1)
    json.dump(traffic, open(os.path.join(os.path.dirname(prefix) or ".", "pmc_traffic.json"), "w"), indent=1)
    json.dump(raw, open(os.path.join(os.path.dirname(prefix) or ".", "pmc_traffic_raw.json"), "w"), indent=1)
    # measured VALU utilisation (tools/prof_valu.sh): rocprof's derived VALUBusy (100 x SQ_ACTIVE_INST_VALU /
    # CU_NUM / GRBM_GUI_ACTIVE: the share of the kernel's time the CUs issue vector ALU instructions) and
    # VALUUtilization (active lanes per VALU instruction), with the raw counters
    valu = {}
    for k, d in per_kernel.items():
        if "VALUBusy" in d or "SQ_INSTS_VALU" in d:
            valu[k] = {n: round(d[n], 3) for n in ("VALUBusy", "VALUUtilization", "SQ_INSTS_VALU",
                                                    "SQ_INSTS_VALU_TRANS_F32", "SQ_ACTIVE_INST_VALU",
                                                    "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")
                       if n in d}
            valu[k]["source"] = "rocprofv3 --pmc VALUBusy VALUUtilization / SQ counters, tools/prof_valu.sh"
    json.dump(valu, open(os.path.join(os.path.dirname(prefix) or ".", "pmc_valu.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
