"""One fp8 GEMM shape x tile config, a few launches (for rocprofv3 --pmc passes)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bioengine_worker_amd.ops.fp8 import Fp8Linear, linear_fp8, quantize_rows  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16448, 2304, 768)))
cfgs = [int(c) for c in (sys.argv[4].split(",") if len(sys.argv) > 4 else ["1"])]
dev = torch.device("cuda")
x = torch.randn(M, K, device=dev).bfloat16()
lin = Fp8Linear(torch.randn(N, K, device=dev) * 0.02, torch.randn(N, device=dev))
xq, sx = quantize_rows(x)
for c in cfgs:
    for _ in range(3):
        linear_fp8(xq, sx, lin.wq, lin.sw, lin.bias, False, tile_cfg=c)
torch.cuda.synchronize()
print("done")
