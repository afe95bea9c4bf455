"""wgrad GEMM variants at the CPSAM fine-tune shapes (m = 8192 tokens): out fp32 [n, k] = dy^T x.
(a) hipBLASLt mm(out_dtype=fp32) (current), (b) split-K bmm(out_dtype=fp32) + sum, (c) rocBLAS backend."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = torch.device("cuda", 0)
    m = 8192
    for n, k in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        dy = torch.randn(m, n, device=dev).bfloat16()
        x = torch.randn(m, k, device=dev).bfloat16()
        out = torch.empty(n, k, device=dev)
        fl = 2 * m * n * k
        res = {"n": n, "k": k, "m": m}
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        res["blt_us"] = round(t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)), 1)
        for S in (2, 4, 8):
            ws = torch.empty(S, n, k, device=dev)

            def sk():
                torch.bmm(dy.view(S, m // S, n).transpose(1, 2), x.view(S, m // S, k), out_dtype=torch.float32, out=ws)
                torch.sum(ws, 0, out=out)
            try:
                res[f"splitk{S}_us"] = round(t(sk), 1)
                sk()
                res[f"splitk{S}_err"] = float((out - ref).abs().max() / ref.abs().max())
            except Exception as e:  # noqa: BLE001
                res[f"splitk{S}_err"] = str(e)[:100]
        try:
            torch.backends.cuda.preferred_blas_library("rocblas")
            res["rocblas_us"] = round(t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)), 1)
        except Exception as e:  # noqa: BLE001
            res["rocblas_err"] = str(e)[:100]
        finally:
            torch.backends.cuda.preferred_blas_library("hipblaslt")
        res["blt_tflops"] = round(fl / res["blt_us"] / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
