#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc ``--save-temps`` .s file, per basic block.

usage: python tools/isa_stats.py FILE.s KERNEL_SUBSTRING [--blocks]
Classes: mfma, ds_read, ds_write, gload, gstore, valu, salu, waitcnt, barrier, branch.
"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_load")):
        return "ds_read"
    if op.startswith(("ds_write", "ds_store")):
        return "ds_write"
    if op.startswith(("global_load", "buffer_load", "flat_load", "s_load", "s_buffer_load")):
        return "gload" if not op.startswith("s_") else "sload"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "gstore"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return op


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN\S*" + re.escape(key) + r"\S*:", l))
    blocks = collections.OrderedDict()
    cur = "entry"
    blocks[cur] = collections.Counter()
    total = collections.Counter()
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or l.strip().startswith(".Lfunc_end"):
            break
        s = l.strip()
        if re.match(r"^\.LBB\S+:", s):
            cur = s.split(":")[0]
            blocks[cur] = collections.Counter()
            continue
        if not s or s.startswith((".", ";")):
            continue
        k = classify(s.split()[0])
        blocks[cur][k] += 1
        total[k] += 1
    print("total", dict(total))
    if "--blocks" in sys.argv:
        for b, c in blocks.items():
            if sum(c.values()):
                print(b, sum(c.values()), dict(c))


if __name__ == "__main__":
    main()
