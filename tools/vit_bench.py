"""ViT kernels on MI355X: flash-attention TFLOP/s and end-to-end DINOv2 ViT-B/14 / Cellpose-SAM throughput,
each against the PyTorch path of the same model (torch SDPA / eager, bf16)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from bioengine_worker_amd.ops.transformer import flash_attention  # noqa: E402


def bench(fn, n=20, warm=3):
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
    for B, N, H in ((64, 257, 12), (8, 1024, 16), (4, 4096, 16)):
        qkv = torch.randn(B, N, 3, H, 64, device=dev).bfloat16()
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        fl = 4.0 * B * H * N * N * 64
        t = bench(lambda: flash_attention(q, k, v))
        qt, kt, vt = (x.transpose(1, 2) for x in (q, k, v))
        ts = bench(lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt))
        print(json.dumps({"attn": [B, N, H], "ms": round(t * 1e3, 3), "TFs": round(fl / t / 1e12, 1),
                          "torch_sdpa_ms": round(ts * 1e3, 3)}), flush=True)
    g = 32
    B, H = 8, 16
    qkv = torch.randn(B, g * g, 3, H, 64, device=dev).bfloat16()
    rh = torch.randn(B, H, g * g, g, device=dev)
    rw = torch.randn(B, H, g * g, g, device=dev)
    t = bench(lambda: flash_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], 0.125, rh, rw))
    print(json.dumps({"attn_relpos": [B, g * g, H], "ms": round(t * 1e3, 3),
                      "TFs": round(4.0 * B * H * (g * g) ** 2 * 64 / t / 1e12, 1)}), flush=True)

    from bioengine_worker_amd.models.vit import ViT, ViTConfig, ViTEngine
    net = ViT(ViTConfig.dinov2("vitb14")).randomize_(0).eval()
    eng = ViTEngine(net, dev)
    x = torch.randn(64, 3, 224, 224, device=dev)
    t = bench(lambda: eng.embed(x), n=10)
    netb = net.to(dev).to(torch.bfloat16)
    with torch.no_grad():
        tr = bench(lambda: netb(x.bfloat16()), n=10)
    print(json.dumps({"dinov2_vitb14_batch64_imgs_per_s": round(64 / t, 1), "ms": round(t * 1e3, 2),
                      "torch_eager_bf16_imgs_per_s": round(64 / tr, 1)}), flush=True)
    del netb, net, eng
    from bioengine_worker_amd.models.cpsam import CPSAM, CPSAMEngine
    net = CPSAM().randomize_(0).eval()
    eng = CPSAMEngine(net, dev)
    x = torch.randn(8, 3, 256, 256, device=dev)
    t = bench(lambda: eng(x), n=5)
    print(json.dumps({"cpsam_vitl8_256px_tiles_per_s": round(8 / t, 1), "ms_batch8": round(t * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
