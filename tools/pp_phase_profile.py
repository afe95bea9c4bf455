#!/usr/bin/env python3
"""Phase profile of the ping-pong level-0 half-blocks (csrc/kernels/conv_pair.hip,
conv_pair_pp_kernel): wave 0 of each of the two wave groups accumulates s_memtime cycles of every
phase's own work and of its wait at the closing workgroup barrier.  The slots pair one group's
MFMA phase with the other's VALU phase, so a phase's wait is the time its partner phase ran longer.

One CPnet forward at the headline batch (288 tiles of 224^2); one JSON line per ping-pong call with
cycles per tile (mean over workgroups and both groups).  Usage: python tools/pp_phase_profile.py"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine  # noqa: E402
from bioengine_worker_amd.ops import _native  # noqa: E402
from bioengine_worker_amd.ops import conv_pair as cp  # noqa: E402


def names(nca):
    ph = []
    for c in range(nca):
        ph += [f"commit{c}", f"stageA{c}"]
    return ph + ["epiA", "stageB", "epiB"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=288)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    net = CPnet().randomize_(0).eval()
    eng = CPnetEngine(net, dev)
    x = torch.randn(args.tiles, 224, 224, 8, device=dev).bfloat16()
    x[..., 2:] = 0
    cap = 1024
    buf = torch.zeros(cap * 32, dtype=torch.int64, device=dev)
    rows = []
    orig_pair, orig_head = cp.conv_pair, getattr(cp, "conv_pair_head", None)

    def collect(tag, xin):
        torch.cuda.synchronize()
        s = buf.view(cap, 2, 16).cpu().double()
        used = s[:, :, 15] > 0
        if not used.any():
            return
        nca = 2 if xin.shape[-1] == 64 else 1
        nm = names(nca)
        out = {"call": tag, "cin": int(xin.shape[-1]), "workgroups": int(used[:, 0].sum())}
        for g in (0, 1):
            sg = s[:, g][used[:, g]]
            it = sg[:, 15]
            out[f"work_g{g}"] = {nm[i]: round(float((sg[:, i] / it).mean())) for i in range(len(nm))}
            out[f"wait_g{g}"] = {nm[i]: round(float((sg[:, 8 + i] / it).mean())) for i in range(len(nm))}
        out["cycles_per_2tiles"] = round(sum(out["work_g0"].values()) + sum(out["wait_g0"].values()))
        rows.append(out)

    def pair(xin, spec, **kw):
        buf.zero_()
        y = orig_pair(xin, spec, **kw)
        collect("pair", xin)
        return y

    def head(xin, *a, **kw):
        buf.zero_()
        y = orig_head(xin, *a, **kw)
        collect("head", xin)
        return y

    with torch.no_grad():
        eng(x)
        torch.cuda.synchronize()
        _native.call("be_conv_pair_pp_set_stamps", _native.ptr(buf), cap)
        cp.conv_pair = pair
        if orig_head is not None:
            cp.conv_pair_head = head
        try:
            eng(x)
        finally:
            cp.conv_pair = orig_pair
            if orig_head is not None:
                cp.conv_pair_head = orig_head
            _native.call("be_conv_pair_pp_set_stamps", None, 0)
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
