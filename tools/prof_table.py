#!/usr/bin/env python3
"""Markdown table of a rocprofv3 ``*_kernel_stats.csv`` (top-N kernels by total time).

    python tools/prof_table.py gpurun_out/prof/bench_kernel_stats.csv [N] [--steps K]
"""
import csv
import sys


def table(path: str, n: int = 20, steps: int | None = None) -> str:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
    calls = sum(int(r["Calls"]) for r in rows)
    out = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:n]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")[:100]
        out.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    foot = f"\nTotal kernel time: {tot:.1f} ms over {calls} launches"
    if steps:
        foot += f" ({tot / steps:.2f} ms and {calls // steps} launches per step over {steps} steps)"
    return "\n".join(out) + foot + "."


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = None
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
        args = [a for a in args if a != str(steps)]
    print(table(args[0], int(args[1]) if len(args) > 1 else 20, steps))
