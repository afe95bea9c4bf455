#!/usr/bin/env python3
"""Per-kernel time over the last K training steps of a rocprofv3 kernel trace.

Steps are delimited by a marker kernel that runs once per step (default: the fused AdamW), so
warm-up, autotuning and graph-capture launches before the window are excluded.  Prints a table
(ms per step, % of the window, calls per step) and the window's kernel-busy ms per step.
Usage: python tools/kt_steps.py <kernel_trace.csv> [--steps 3] [--marker adamw_kernel] [--top 30]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    pat = re.compile(a.marker)
    marks = [i for i, r in enumerate(rows) if pat.search(r[2])]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
    win = rows[lo:hi]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[n][0] += e - s
        agg[n][1] += 1
    tot = sum(v[0] for v in agg.values())
    wall = win[-1][1] - win[0][0]
    print(f"window: {a.steps} steps, kernel-busy {tot / a.steps / 1e6:.3f} ms/step, wall {wall / a.steps / 1e6:.3f} ms/step")
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{d / a.steps / 1e6:8.3f} ms {100 * d / tot:5.1f}% {c / a.steps:6.1f}/step  {n[: a.width]}")


if __name__ == "__main__":
    main()
