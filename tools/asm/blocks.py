"""Split one kernel of a gfx950 .s file into basic blocks and count instruction classes per block.

  python tools/asm/blocks.py file.s kernel_substring [top_n]
"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        l = l.split(";")[0].rstrip()
        if start is None and l.endswith(":") and sub in l and not l.startswith(".") and not l.startswith("\t"):
            start = i
        elif start is not None and (l.startswith("\t.section") or l.startswith(".Lfunc_end")):
            return lines[start:i]
    return lines[start:] if start is not None else []


def classify(op):
    if op.startswith("v_exp") or op.startswith("v_rcp") or op.startswith("v_log") or op.startswith("v_sqrt") or op.startswith("v_rsq"):
        return "trans"
    if op.startswith("v_pk_"):
        return "vpk"
    if op.startswith("v_cmp") or op.startswith("v_cmpx"):
        return "vcmp"
    if op.startswith("v_cndmask"):
        return "vsel"
    if op.startswith("v_permlane") or "dpp" in op:
        return "vperm"
    if op.startswith("v_mov") or op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("v_writelane"):
        return "vmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    lines = kernel_lines(path, sub)
    blocks, cur, name = [], Counter(), "entry"
    for l in lines:
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if re.match(r"^\.LBB\d+_\d+:", s):
                blocks.append((name, cur))
                name, cur = s[:-1], Counter()
            continue
        op = s.split()[0]
        if op.endswith(":"):
            continue
        cur[classify(op + (" dpp" if "row_" in s or "quad_perm" in s else ""))] += 1
        cur["_total"] += 1
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            pass
    blocks.append((name, cur))
    blocks.sort(key=lambda b: -b[1]["_total"])
    keys = ["_total", "vpk", "valu", "trans", "vcmp", "vsel", "vperm", "vmov", "salu", "lds", "vmem", "wait"]
    print("block".ljust(14) + "".join(k[:6].rjust(7) for k in keys))
    for n, c in blocks[:top]:
        print(n.ljust(14) + "".join(str(c[k]).rjust(7) for k in keys))


if __name__ == "__main__":
    main()
