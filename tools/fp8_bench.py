"""FP8 GEMM microbench on the DINOv2 ViT-B/14 batch-64 linear shapes (M = 64 x 257 tokens):
HIP block-scaled MFMA GEMM (``be_gemm_fp8``) vs hipBLASLt bf16 (``F.linear``) and, when this
PyTorch build exposes it, hipBLASLt fp8 (``torch._scaled_mm``).  Then the end-to-end ViT-B/14
embedding throughput in bf16 and fp8.  One JSON line per measurement."""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from bioengine_worker_amd.ops.fp8 import FP8_DTYPE, Fp8Linear, linear_fp8, quantize_rows  # noqa: E402


def bench(fn, n=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    M = 64 * 257
    for name, N, K, gelu in (("qkv", 2304, 768, False), ("proj", 768, 768, False), ("fc1", 3072, 768, True),
                             ("fc2", 768, 3072, False), ("sq4096", 4096, 4096, False)):
        Mi = 4096 if name == "sq4096" else M
        x = torch.randn(Mi, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev) * 0.02
        b = torch.randn(N, device=dev)
        lin = Fp8Linear(w, b)
        xq, sx = quantize_rows(x)
        fl = 2.0 * Mi * N * K
        t8 = bench(lambda: linear_fp8(xq, sx, lin.wq, lin.sw, lin.bias, gelu))
        tcfg = {c: round(fl / bench(lambda: linear_fp8(xq, sx, lin.wq, lin.sw, lin.bias, gelu, tile_cfg=c)) / 1e12, 1)
                for c in (1, 2, 3, 4, 5, 6)}
        tq = bench(lambda: quantize_rows(x))
        tqg = bench(lambda: quantize_rows(x, gelu=True))
        wb, bb = w.bfloat16(), b.bfloat16()
        tb = bench(lambda: F.linear(x, wb, bb))
        row = {"gemm": name, "M": Mi, "N": N, "K": K, "gelu": gelu, "hip_fp8_us": round(t8 * 1e6, 1),
               "hip_fp8_TFs": round(fl / t8 / 1e12, 1), "hip_fp8_TFs_by_tile_cfg": tcfg, "quant_us": round(tq * 1e6, 1), "gelu_quant_us": round(tqg * 1e6, 1),
               "hipblaslt_bf16_us": round(tb * 1e6, 1), "hipblaslt_bf16_TFs": round(fl / tb / 1e12, 1)}
        try:
            wt = lin.wq.t()
            one = torch.ones((), device=dev)
            ts = bench(lambda: torch._scaled_mm(xq, wt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
            row["hipblaslt_fp8_us"] = round(ts * 1e6, 1)
            row["hipblaslt_fp8_TFs"] = round(fl / ts / 1e12, 1)
        except Exception as e:  # not every build has fp8 hipBLASLt for gfx950
            row["hipblaslt_fp8"] = f"{type(e).__name__}: {str(e)[:80]}"
        try:  # row-wise scales (the same per-token x per-channel scaling as the HIP kernel)
            sa, sb = sx.reshape(-1, 1).contiguous(), lin.sw.reshape(1, -1).contiguous()
            ts = bench(lambda: torch._scaled_mm(xq, lin.wq.t(), scale_a=sa, scale_b=sb, bias=bb,
                                                out_dtype=torch.bfloat16))
            row["hipblaslt_fp8_rowwise_us"] = round(ts * 1e6, 1)
        except Exception as e:
            row["hipblaslt_fp8_rowwise"] = f"{type(e).__name__}: {str(e)[:80]}"
        print(json.dumps(row), flush=True)

    from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine
    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    x = torch.randn(64, 3, 224, 224, device=dev)
    out = {}
    embs = {}
    for prec in ("bf16", "fp8", "fp8hip"):
        eng = ViTEngine(net, dev, precision=prec[:3] if prec != "bf16" else prec,
                        fp8_gemm="hip" if prec == "fp8hip" else "hipblaslt")
        t = bench(lambda: eng.embed(x), n=10, warm=3)
        out[f"dinov2_vitb14_batch64_{prec}_imgs_per_s"] = round(64 / t, 1)
        out[f"{prec}_ms"] = round(t * 1e3, 3)
        embs[prec] = eng.embed(x)
        del eng
    out["fp8_vs_bf16_cos_min"] = round(F.cosine_similarity(embs["fp8"], embs["bf16"], dim=1).min().item(), 5)
    out["fp8hip_vs_bf16_cos_min"] = round(F.cosine_similarity(embs["fp8hip"], embs["bf16"], dim=1).min().item(), 5)
    out["reference_a100_fp16_imgs_per_s"] = 500.0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
