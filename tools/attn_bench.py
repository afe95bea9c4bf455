"""Micro-benchmark of the CPSAM attention kernels at the fine-tune shape (B=8 crops of 256^2 / patch 8
-> N=1024 tokens, 16 heads, head_dim 64, SAM rel-pos bias): forward and backward (dq + dkv kernels)
timed with HIP events; prints one JSON line per case.  Used for the attention roofline in profiles/."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bioengine_worker_amd.ops import _native, vit_train as vt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bias", type=int, default=1)
    a = ap.parse_args()
    _native.hip()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, H, N, D = a.B, a.H, a.N, 64
    qkv = (torch.randn(B, N, 3, H, D, device=dev) * 0.5).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    rh = rw = None
    if a.bias:
        rh = torch.randn(B, H, N, N // 32, device=dev) * 0.5
        rw = torch.randn(B, H, N, 32, device=dev) * 0.5
    scale = D ** -0.5
    do = (torch.randn(B, N, H, D, device=dev) * 0.5).bfloat16()
    o, lse = vt.attn_fwd(q, k, v, scale, rh, rw)
    for _ in range(3):
        vt.attn_fwd(q, k, v, scale, rh, rw)
        vt.attn_bwd(q, k, v, o, do, lse, scale, rh, rw)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    for _ in range(a.iters):
        vt.attn_fwd(q, k, v, scale, rh, rw)
    ev[1].record()
    for _ in range(a.iters):
        vt.attn_bwd(q, k, v, o, do, lse, scale, rh, rw)
    ev[2].record()
    torch.cuda.synchronize()
    fwd = ev[0].elapsed_time(ev[1]) / a.iters
    bwd = ev[1].elapsed_time(ev[2]) / a.iters
    bh = B * H
    ffl, bfl = 4 * N * N * D * bh, 14 * N * N * D * bh  # bwd: dq kernel 6 + dkv kernel 8 (recompute incl.)
    print(json.dumps({"B": B, "H": H, "N": N, "bias": bool(a.bias), "fwd_ms": round(fwd, 4),
                      "fwd_tflops": round(ffl / fwd / 1e9, 1), "bwd_ms": round(bwd, 4),
                      "bwd_tflops": round(bfl / bwd / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
