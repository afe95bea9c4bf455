#!/usr/bin/env python3
"""Validate every hipBLASLt heuristic candidate of the fused GEMMs against an fp32 reference (the
autotuner must only ever pick correct kernels): one JSON line per (op, candidate index)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bioengine_worker_amd.ops import _native, gemm  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M, D, F4 = 2048, 1024, 4096
    bf = dict(device=dev, dtype=torch.bfloat16)
    dm, w2 = torch.randn(M, D, **bf), (torch.randn(D, F4, device=dev) * F4 ** -0.5).bfloat16()
    f = torch.randn(M, F4, **bf)
    ff = f.float().requires_grad_(True)
    (gp,) = torch.autograd.grad(F.gelu(ff, approximate="tanh"), ff, grad_outputs=dm.float() @ w2.float())
    x, w, b = torch.randn(M, D, **bf), (torch.randn(F4, D, device=dev) * D ** -0.5).bfloat16(), torch.randn(F4, **bf)
    ref_lin = F.linear(x.float(), w.float(), b.float())
    ref_wg = dm.float().t() @ x.float()
    lib = _native.hip()
    for i in range(32):
        lib.be_lt_reset(i)
        db = torch.zeros(F4, device=dev)
        df = gemm.mm_dgelu(dm, w2, f, out_db=db)
        y = gemm.linear(x, w, b)
        out = torch.empty(D, D, device=dev)
        gemm.wgrad(dm, x, out)
        torch.cuda.synchronize()
        pl = {(r["epi"], r["fp32_out"]): (r["candidates"], r["rejected"]) for r in gemm.plans()}
        print(json.dumps({"cand": i, "dgelu_rel": round(rel(df, gp), 5), "bgrad_rel": round(rel(db, gp.sum(0)), 5),
                          "linear_bias_rel": round(rel(y, ref_lin), 5), "wgrad_rel": round(rel(out, ref_wg), 6),
                          "n_cand": {f"{k[0]}/{k[1]}": v for k, v in pl.items()}}), flush=True)
    lib.be_lt_reset(-1)  # the autotuner itself: it must reject the wrong candidates
    db = torch.zeros(F4, device=dev)
    df = gemm.mm_dgelu(dm, w2, f, out_db=db)
    torch.cuda.synchronize()
    print(json.dumps({"cand": "tuned", "dgelu_rel": round(rel(df, gp), 5), "bgrad_rel": round(rel(db, gp.sum(0)), 5),
                      "plans": gemm.plans()}), flush=True)


if __name__ == "__main__":
    main()
