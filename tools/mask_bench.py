#!/usr/bin/env python3
"""Mask-recovery stage in isolation (the headline's network output for 32 512x512 images, or the
cell-like synthetic flows): times ``compute_masks_gpu`` and its flow-QC diffusion per sweep
variant (``BE_DIFFUSE_VARIANT``), interleaved in one process so box-to-box variance cancels."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2",
                    help="BE_DIFFUSE_VARIANT values, dv8,dv4,.. for BE_DIFFUSE_DV, q1 / q0 (diffusion queue), fw1 / fw0 (one-wave fill), "
                         "fe:<entry> (follow-flows launch), base (all defaults), r04 (the round-4 stage)")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from bioengine_worker_amd.cellpose import gpu as cg
    from bioengine_worker_amd.cellpose.gpu import compute_masks_gpu, follow_and_label, masks_to_flows_gpu
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells

    dev = torch.device("cuda", 0)
    runner = CellposeRunner(device=dev, seed=0)
    imgs = torch.from_numpy(synthetic_cells(32, 512, 512, nchan=2, seed=0)).to(dev)
    _, y, _ = runner.eval(imgs, EvalParams(compute_masks=False))
    y = y.float().contiguous()
    M = follow_and_label(y, 200, 0.0, 0.4)
    if isinstance(M, tuple):
        M = M[0]
    ref = None
    res = {}
    for rep in range(a.reps + 1):
        for v in a.variants.split(","):
            if v.startswith("dv"):
                os.environ["BE_DIFFUSE_DV"] = v[2:]
            elif v.startswith("q"):
                cg.DIFFUSE_QUEUE = v[1:] == "1"
            elif v.startswith("fw"):
                cg.FILL_WAVE = v[2:] == "1"
            elif v.startswith("fe:"):
                cg.FOLLOW_FLOWS_ENTRY = v[3:]
            elif v == "base":  # every default on
                cg.DIFFUSE_QUEUE, cg.FILL_WAVE, cg.FOLLOW_FLOWS_ENTRY = True, True, "be_cp_follow_flows_lds"
            elif v == "r04":  # the round-4 mask stage
                cg.DIFFUSE_QUEUE, cg.FILL_WAVE, cg.FOLLOW_FLOWS_ENTRY = False, False, "be_cp_follow_flows_xcd"
            else:
                os.environ["BE_DIFFUSE_VARIANT"] = v
            torch.cuda.synchronize()
            t = time.perf_counter()
            mu, err, _ = masks_to_flows_gpu(M, dp=y)
            torch.cuda.synchronize()
            t_qc = time.perf_counter() - t
            t = time.perf_counter()
            masks = compute_masks_gpu(y, 200, 0.0, 0.4, 15, 0.4)
            torch.cuda.synchronize()
            t_all = time.perf_counter() - t
            if ref is None:
                ref = (mu, err, masks)
            diff = {"mu_max_abs": float((mu - ref[0]).abs().max()),
                    "mu_frac_gt_1e-3": float(((mu - ref[0]).abs() > 1e-3).float().mean()),
                    "err_rel": float((err - ref[1]).abs().max() / ref[1].abs().max().clamp_min(1e-12)),
                    "masks_equal": bool(torch.equal(masks, ref[2]))}
            if rep:
                res.setdefault(v, []).append((t_qc * 1e3, t_all * 1e3, diff))
    for v, ts in res.items():
        qc = sorted(t[0] for t in ts)[len(ts) // 2]
        al = sorted(t[1] for t in ts)[len(ts) // 2]
        print(json.dumps({"variant": v, "masks_to_flows_ms": round(qc, 3), "compute_masks_ms": round(al, 3),
                          "labels": int(M.max()), "vs_variant0": ts[-1][2]}), flush=True)


if __name__ == "__main__":
    main()
