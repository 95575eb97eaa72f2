"""Instruction mix of one kernel in a hipcc --save-temps .s file (tools only).

usage: python tools/isa_stats.py FILE.s NAME_SUBSTRING [--blocks]
Prints VALU / SALU / LDS / VMEM / branch counts for the whole kernel and, with
--blocks, per basic block (label), so loop bodies can be read off directly.
"""
from __future__ import annotations

import re
import sys
from collections import Counter


def cat(op: str) -> str:
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "br"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    txt = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):.*?\n(.*?)^\s*s_endpgm", txt, re.S | re.M)
    if not m:
        sys.exit(f"no kernel matching {name}")
    print(m.group(1))
    total = Counter()
    blocks = []
    cur = ("entry", Counter())
    for raw in m.group(2).split("\n"):
        ln = raw.split(";")[0].strip()
        if ln.endswith(":"):
            blocks.append(cur)
            cur = (ln[:-1], Counter())
            continue
        if not ln or ln.startswith("."):
            continue
        c = cat(ln.split()[0])
        total[c] += 1
        cur[1][c] += 1
    blocks.append(cur)
    print("total", dict(total))
    if "--blocks" in sys.argv:
        for lab, c in blocks:
            if sum(c.values()):
                print(f"  {lab:24s} {dict(c)}")


if __name__ == "__main__":
    main()
