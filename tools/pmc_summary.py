#!/usr/bin/env python3
"""Summarise a ``rocprofv3 --pmc ... --kernel-trace --output-format csv`` run: per kernel, every
counter summed over the kernel's dispatches plus its ratio to ``SQ_WAVE_CYCLES`` (the per-wave-cycle
rates that compare kernels of different sizes: MFMA-busy, LDS conflicts per LDS instruction, waits).

    python tools/pmc_summary.py gpurun_out/r04/pmc/pairs/p_counter_collection.csv [--match conv] [--top 8]
"""
import argparse
import collections
import csv


def summarise(path: str, match: str = "", top: int = 8) -> str:
    sums: dict = collections.defaultdict(lambda: collections.defaultdict(float))
    disp: dict = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    order = sorted(sums, key=lambda k: -sums[k].get("SQ_WAVE_CYCLES", 0.0))[:top]
    out = ["# rocprofv3 --pmc, summed over the kernel's dispatches; ratios are per SQ_WAVE_CYCLES"]
    for k in order:
        c = sums[k]
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out.append(f"{k[:160]}  ({len(disp[k])} dispatches)")
        for n in sorted(c):
            out.append(f"  {n:<32} {c[n]:>14.0f}  ratio {c[n] / wc:.3f}")
        if c.get("SQ_INSTS_LDS"):
            out.append(f"  LDS bank conflicts / LDS inst      {c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_INSTS_LDS']:.2f}")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    print(summarise(a.csv, a.match, a.top))


if __name__ == "__main__":
    main()
