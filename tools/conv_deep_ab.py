#!/usr/bin/env python3
"""A/B of the per-layer conv kernel options on the headline CPnet's deep layers (3x3, Cin >= 64):
every recorded fused_conv2d call of one 32-image batch is replayed with nw = 4 and nw = 8 (HIP-event
median of --reps launches).  Run once per kernel library (BE_HIP_LIB) to compare builds.
Prints one JSON line per (layer, nw) and a per-nw total."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.conv_roofline import describe, record_calls  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--nw", default="4,8")
    ap.add_argument("--all", action="store_true", help="every layer, not only the deep 3x3 ones")
    a = ap.parse_args()
    from bioengine_worker_amd.ops import conv as convops

    dev = torch.device("cuda", 0)
    calls = record_calls(dev)
    tot = {}
    for i, (x, pc, kw) in enumerate(calls):
        if not a.all and not (pc.ks == 3 and pc.cin_pad >= 64):
            continue
        name, flops, _ = describe(x, pc, kw)
        for nw in [int(v) for v in a.nw.split(",")]:
            if kw.get("x2") is not None and nw == 8:
                continue
            ts = []
            for r in range(a.reps + 3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                convops.fused_conv2d(x, pc, nw=nw or None, **kw)  # nw 0 = the shape policy
                e.record()
                e.synchronize()
                if r >= 3:
                    ts.append(s.elapsed_time(e))
            ms = sorted(ts)[len(ts) // 2]
            tot[nw] = tot.get(nw, 0.0) + ms
            print(json.dumps({"idx": i, "layer": name, "nw": nw, "ms": round(ms, 4),
                              "TFs": round(flops / ms / 1e9, 1), "lib": os.path.basename(os.path.dirname(
                                  os.environ.get("BE_HIP_LIB", "main/x")))}), flush=True)
    print(json.dumps({"total_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
