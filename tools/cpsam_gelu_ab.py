"""A/B: Cellpose-SAM inference lin1 + bias + GELU as hipBLASLt GEMM + the HIP bias_gelu_ pass ("lib")
against hipBLASLt's fused GELU_BIAS epilogue ("ltgelu", tanh-approximated GELU).  One process,
alternating arms; prints per-arm forward ms over 72 tiles (8 images x 9 tiles of 256^2) and the
output cosine / max-abs difference against the lib arm."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bioengine_worker_amd.models.cpsam import CPSAM, CPSAMEngine


def bench(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    net = CPSAM().randomize_(0).eval()
    eng = CPSAMEngine(net, dev)
    x = torch.randn(72, 3, 256, 256, device=dev)
    outs = {}
    for arm in ("lib", "ltgelu"):
        eng.GEMM = arm
        outs[arm] = eng(x).float()
    ref = outs["lib"]
    d = outs["ltgelu"]
    cos = torch.nn.functional.cosine_similarity(ref.flatten(), d.flatten(), dim=0).item()
    print(json.dumps({"cosine_ltgelu_vs_lib": round(cos, 6), "max_abs": round((ref - d).abs().max().item(), 4),
                      "ref_absmax": round(ref.abs().max().item(), 3)}), flush=True)
    res = {"lib": [], "ltgelu": []}
    for rep in range(3):
        for arm in ("lib", "ltgelu"):
            eng.GEMM = arm
            res[arm].append(bench(lambda: eng(x)) * 1e3)
    for arm, v in res.items():
        print(json.dumps({"arm": arm, "ms_72_tiles": [round(t, 2) for t in v], "tiles_per_s": round(72e3 / min(v), 1)}),
              flush=True)


if __name__ == "__main__":
    main()
