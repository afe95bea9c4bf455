#!/usr/bin/env python3
"""Which hipBLASLt epilogue / layout / type combinations this build supports at the ViT MLP shapes:
one JSON line per combination with the be_lt_gemm status (0 = ran)."""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bioengine_worker_amd.ops import _native, gemm  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M, K, N = int(os.environ.get("M", 2048)), 1024, 4096
    bf = dict(device=dev, dtype=torch.bfloat16)
    X = torch.randn(M * max(K, N), **bf)
    Y = torch.randn(max(K, N) * max(K, N), **bf)
    D = torch.empty(M * N * 2, device=dev, dtype=torch.float32)
    aux = torch.randn(M * N, **bf)
    bias16 = torch.randn(N, **bf)
    bias32 = torch.randn(N, device=dev)
    ws = gemm._workspace(dev)
    names = {1: "BIAS", 2: "GELU_AUX_BIAS", 3: "DGELU_BGRAD", 4: "GELU_BIAS", 5: "BGRADB", 6: "DGELU"}
    epis = [int(e) for e in os.environ.get("EPIS", "1,2,3,4,5,6").split(",")]
    for epi, (tx, ty), flags in itertools.product(epis, [(0, 1), (0, 0), (1, 0)], range(8)):
        b = bias32 if flags & 1 else bias16
        fn = _native.hip().be_lt_gemm
        rc = fn(_native.ptr(X), _native.ptr(Y), _native.ptr(D), _native.ptr(b), _native.ptr(aux), _native.ptr(b),
                _native.ptr(ws), ws.numel(), M, N, K, tx, ty, 0, epi, flags, 1.0, 0.0, _native.stream(dev))
        torch.cuda.synchronize()
        print(json.dumps({"M": M, "epi": names[epi], "tx": tx, "ty": ty, "bias_fp32": flags & 1, "aux_type_default": bool(flags & 2),
                          "bias_type_default": bool(flags & 4), "rc": rc}), flush=True)


if __name__ == "__main__":
    main()
