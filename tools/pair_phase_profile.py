#!/usr/bin/env python3
"""Where a fused CPnet half-block (csrc/kernels/conv_pair.hip) spends its time, phase by phase.

The level-0/1 half-blocks of one CPnet forward at the headline batch (288 tiles of 224^2) are run
through the phase-stamped build of the kernel (``be_conv_pair_set_stamps``): wave 0 of every
workgroup accumulates ``s_memtime`` deltas over its tiles for

  halo commit (input halo registers -> activated LDS image, incl. the barriers around it),
  stage-A MFMA (issue of the next tile's halo loads + the h-region implicit GEMM),
  stage-A epilogue (actB + skip -> h in LDS, incl. the barrier before it),
  stage-B MFMA (barrier + the output implicit GEMM),
  output epilogue (barrier, bias + residual, staged 16-byte stores).

Prints one JSON line per half-block call: cycles per tile in each phase (mean over workgroups)
and their shares.  Diagnostic only: the stamped build runs ~1 % slower than the production one.
Usage: ``python tools/pair_phase_profile.py [--tiles 288]``.
"""
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

PHASES = ("halo_commit", "stageA_mfma", "stageA_epi", "stageB_mfma", "out_epi")


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
    buf = torch.zeros(cap * 8, dtype=torch.int64, device=dev)
    rows = []
    orig = cp.conv_pair

    def stamped(xin, spec, **kw):
        buf.zero_()
        y = orig(xin, spec, **kw)
        torch.cuda.synchronize()
        s = buf.view(cap, 8).cpu()
        used = s[:, 7] > 0
        if used.any():
            s = s[used].double()
            tiles = s[:, 7]
            per_tile = {p: float((s[:, i] / tiles).mean()) for i, p in enumerate(PHASES)}
            tot = sum(per_tile.values())
            rows.append({"cin": int(xin.shape[-1]), "cm": int(spec.pb.cout),
                         "in_hw": list(xin.shape[1:3]), "inmode": spec.inmode, "x2": kw.get("x2") is not None,
                         "res_mode": kw.get("res_mode", "none"), "workgroups": int(used.sum()),
                         "tiles_per_wg": float(tiles.mean()),
                         "cycles_per_tile": {k: round(v) for k, v in per_tile.items()},
                         "share": {k: round(v / tot, 3) for k, v in per_tile.items()}})
        return y

    with torch.no_grad():
        eng(x)  # warm-up (allocator, kernels) on the production build
        torch.cuda.synchronize()
        _native.call("be_conv_pair_set_stamps", _native.ptr(buf), cap)
        cp.conv_pair = stamped
        try:
            eng(x)
        finally:
            cp.conv_pair = orig
            _native.call("be_conv_pair_set_stamps", None, 0)
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
