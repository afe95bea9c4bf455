#!/usr/bin/env python3
"""Aggregate Chrome-trace JSON files written by ``profiling/trace.py``: per span name -> count,
total / mean wall ms (and device ms for the "gpu" track).  Usage: ``python tools/trace_summary.py f1.json ...``."""
import collections
import json
import sys


def summarize(paths):
    agg = collections.defaultdict(lambda: [0, 0.0, []])
    for p in paths:
        for e in json.load(open(p))["traceEvents"]:
            if e.get("ph") != "X":
                continue
            k = ("gpu:" if e.get("cat") == "gpu" else "") + e["name"]
            agg[k][0] += 1
            agg[k][1] += e["dur"] / 1e3
            agg[k][2].append(e["dur"] / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    return [{"span": k, "count": n, "total_ms": round(t, 2), "mean_ms": round(t / n, 3),
             "p50_ms": round(sorted(d)[len(d) // 2], 3)} for k, (n, t, d) in rows]


if __name__ == "__main__":
    for r in summarize(sys.argv[1:]):
        print(json.dumps(r))
