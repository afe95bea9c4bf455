#!/usr/bin/env python3
"""Per-layer roofline of the headline CPnet forward.

Records every fused conv the inference engine launches for one batch of 32 512x512 images
(288 tiles of 224x224), then replays each call in isolation:

* ``--mode time``: median of 20 HIP-event-timed launches per layer -> ms, TFLOP/s (true Cin, not
  the padded one) and the layer's minimum HBM traffic (input once -- 4x for a pooling loader,
  1/4 for an upsampling one -- + skip input + residual + output) in GB/s, against the MI355X
  dense-bf16 roof (2.5 PFLOP/s) and HBM roof (8 TB/s).
* ``--mode pmc``: every layer once after a warm-up round, for ``rocprofv3 --pmc`` passes; the
  dispatch order is written to ``--order`` so the counter rows can be mapped back to layers
  (``tools/conv_roofline_table.py``).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PEAK_TF, PEAK_GBS = 2500.0, 8000.0


def record_calls(dev):
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells
    from bioengine_worker_amd.ops import conv as convops

    runner = CellposeRunner(device=dev, seed=0)
    imgs = torch.from_numpy(synthetic_cells(32, 512, 512, nchan=2, seed=0)).to(dev)
    p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15)
    runner.eval(imgs, p)
    calls = []
    orig = convops.fused_conv2d

    def spy(x, pc, **kw):
        out = orig(x, pc, **kw)
        calls.append((x, pc, dict(kw)))
        return out

    convops.fused_conv2d = spy
    try:
        runner.eval(imgs, EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15,
                                     compute_masks=False))
    finally:
        convops.fused_conv2d = orig
    torch.cuda.synchronize()
    return calls


def describe(x, pc, kw):
    N, Hs, Ws, Cin = x.shape
    mode = kw.get("inmode", "none")
    H, W = {"none": (Hs, Ws), "up2": (2 * Hs, 2 * Ws), "pool2": (Hs // 2, Ws // 2)}[mode]
    cin, cout = pc.cin, (kw.get("cout_valid") or pc.cout)
    flops = 2.0 * N * H * W * cout * cin * pc.ks * pc.ks
    byt = x.numel() * 2 + N * H * W * cout * (4 if kw.get("out_nchw_f32") else 2)
    if kw.get("x2") is not None:
        byt += kw["x2"].numel() * 2
    if kw.get("residual") is not None:
        byt += kw["residual"].numel() * 2
    name = f"{pc.ks}x{pc.ks} {cin}->{cout} @{H}x{W}" + ("" if mode == "none" else f" {mode}") + \
        (" +skip" if kw.get("x2") is not None else "") + (" +res" if kw.get("residual") is not None else "") + \
        (" f32-head" if kw.get("out_nchw_f32") else "")
    return name, flops, byt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="time", choices=["time", "pmc"])
    ap.add_argument("--order", default="gpurun_out/conv_roofline_order.json")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from bioengine_worker_amd.ops import conv as convops

    dev = torch.device("cuda", 0)
    calls = record_calls(dev)
    if a.mode == "pmc":
        for x, pc, kw in calls:  # warm-up round
            convops.fused_conv2d(x, pc, **kw)
        torch.cuda.synchronize()
        order = []
        for i, (x, pc, kw) in enumerate(calls):
            convops.fused_conv2d(x, pc, **kw)
            torch.cuda.synchronize()
            order.append(dict(zip(("layer", "flops", "bytes"), describe(x, pc, kw)), idx=i))
        os.makedirs(os.path.dirname(a.order) or ".", exist_ok=True)
        json.dump(order, open(a.order, "w"))
        print(f"pmc replay: {len(calls)} layers", flush=True)
        return
    tot_ms = tot_f = 0.0
    for i, (x, pc, kw) in enumerate(calls):
        name, flops, byt = describe(x, pc, kw)
        ts = []
        for r in range(a.reps + 3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            convops.fused_conv2d(x, pc, **kw)
            e.record()
            e.synchronize()
            if r >= 3:
                ts.append(s.elapsed_time(e))
        ms = sorted(ts)[len(ts) // 2]
        tf, gbs = flops / ms / 1e9, byt / ms / 1e6
        t_roof = max(flops / (PEAK_TF * 1e12), byt / (PEAK_GBS * 1e9)) * 1e3
        tot_ms += ms
        tot_f += flops
        print(json.dumps({"idx": i, "layer": name, "ms": round(ms, 4), "TFs": round(tf, 1), "GBs": round(gbs, 1),
                          "pct_mfma_peak": round(100 * tf / PEAK_TF, 1), "pct_hbm_peak": round(100 * gbs / PEAK_GBS, 1),
                          "bound": "compute" if flops / byt > PEAK_TF * 1e12 / (PEAK_GBS * 1e9) else "memory",
                          "roof_ms": round(t_roof, 4), "x_roof": round(ms / t_roof, 2)}), flush=True)
    print(json.dumps({"total_conv_ms": round(tot_ms, 3), "total_TFLOP": round(tot_f / 1e12, 3),
                      "avg_TFs": round(tot_f / tot_ms / 1e9, 1), "layers": len(calls)}), flush=True)


if __name__ == "__main__":
    main()
