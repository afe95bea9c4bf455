#!/usr/bin/env python3
"""Join ``conv_roofline.py --mode time`` output with the rocprofv3 --pmc passes of
``--mode pmc`` into the per-layer roofline table (markdown).

Usage: conv_roofline_table.py TIME.jsonl ORDER.json PMC_DIR [PMC_DIR ...] > table.md
Each PMC_DIR holds one pass's ``*counter_collection.csv``.  Conv dispatches are matched to layers
by order (the last len(ORDER) conv dispatches of each pass are the measured round)."""
import collections
import csv
import glob
import json
import re
import sys


def pmc_rows(d, n):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        return []
    per = collections.OrderedDict()
    for r in csv.DictReader(open(files[0])):
        if "conv2d_nhwc" not in r.get("Kernel_Name", ""):
            continue
        key = int(r["Dispatch_Id"])
        per.setdefault(key, {"kernel": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = [per[k] for k in sorted(per)]
    return rows[-n:]


def main():
    timed = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"idx"')]
    order = json.load(open(sys.argv[2]))
    n = len(order)
    merged = [dict() for _ in range(n)]
    for d in sys.argv[3:]:
        for i, r in enumerate(pmc_rows(d, n)):
            merged[i].update(r)
    print("| # | layer | kernel | ms | TFLOP/s | % MFMA peak | min-bytes GB/s | L2 fetch GB/s | L2 write GB/s | % HBM peak (fetch+write) | bound | x roofline | wait_any | wait_inst | active |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    tot = 0.0
    for t, m in zip(timed, merged):
        ms = t["ms"]
        tot += ms
        fetch = m.get("FETCH_SIZE")
        write = m.get("WRITE_SIZE")
        fgb = f"{fetch * 1024 / ms / 1e6:.0f}" if fetch else "-"
        wgb = f"{write * 1024 / ms / 1e6:.0f}" if write else "-"
        hbm = f"{100 * ((fetch or 0) + (write or 0)) * 1024 / ms / 1e6 / 8000:.0f}" if fetch and write else "-"
        wc = m.get("SQ_WAVE_CYCLES")
        fr = (lambda k: f"{m[k] / wc:.2f}" if wc and k in m else "-")
        mk = re.search(r"conv2d_nhwc_\w+<[^>]*>", m.get("kernel", ""))
        kern = mk.group(0) if mk else "-"
        print(f"| {t['idx']} | {t['layer']} | `{kern}` | {ms:.3f} | {t['TFs']:.0f} | {t['pct_mfma_peak']:.0f} | {t['GBs']:.0f} | "
              f"{fgb} | {wgb} | {hbm} | {t['bound']} | {t['x_roof']:.1f} | {fr('SQ_WAIT_ANY')} | {fr('SQ_WAIT_INST_ANY')} | "
              f"{fr('SQ_ACTIVE_INST_ANY')} |")
    print(f"\nTotal conv time {tot:.2f} ms over {n} layers.")


if __name__ == "__main__":
    main()
