#!/usr/bin/env python3
"""Batch-1 timeline from a rocprofv3 kernel trace of tools/latency_b1.py: per iteration (delimited by
a marker kernel) the wall span, kernel-busy time, and the largest idle gaps between kernels with the
kernels on either side, so host-side stalls (syncs, launches) show up next to the GPU work.
Usage: python tools/b1_timeline.py <kernel_trace.csv> [--marker tiles_gather_kernel] [--iters 3]"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="tiles_gather_kernel", help="a kernel that runs once per iteration")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    pat = re.compile(a.marker)
    starts = [i for i, r in enumerate(rows) if pat.search(r[2])]
    if len(starts) < a.iters + 1:
        raise SystemExit(f"only {len(starts)} iterations found")
    for s, e in zip(starts[-a.iters - 1:-1], starts[-a.iters:]):
        win = rows[s:e]
        end = max(r[1] for r in win)
        wall = end - win[0][0]
        # busy = union of kernel intervals
        busy, cs, ce = 0, win[0][0], win[0][1]
        for st, en, _ in win[1:]:
            if st > ce:
                busy += ce - cs
                cs, ce = st, en
            else:
                ce = max(ce, en)
        busy += ce - cs
        print(f"iteration: wall {wall / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us, {len(win)} kernels")
        gaps = []
        last_end = win[0][1]
        for i in range(1, len(win)):
            g = win[i][0] - last_end
            if g > 0:
                gaps.append((g, win[i - 1][2][:60], win[i][2][:60], (win[i][0] - win[0][0]) / 1e3))
            last_end = max(last_end, win[i][1])
        for g, before, after, at in sorted(gaps, reverse=True)[: a.gaps]:
            print(f"   gap {g / 1e3:7.1f} us at {at:7.1f} us: {before} -> {after}")
        names = {}
        for st, en, n in win:
            names[n[:70]] = names.get(n[:70], 0) + en - st
        for n, d in sorted(names.items(), key=lambda kv: -kv[1])[:15]:
            print(f"   {d / 1e3:7.1f} us  {n}")


if __name__ == "__main__":
    main()
