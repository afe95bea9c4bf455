#!/usr/bin/env python3
"""Which E8M0 block scale does v_mfma_scale_f32_16x16x128_f8f6f4 apply to which K element, given the
kernel's fragment layout (lane l: row l & 15, K bytes [32 (l >> 4), +32))?  X = ones, W = identity,
per-(row, 32-block) scales s[m, b] = 127 + ((m + 3 b) % 8): y[m, n] = 2^(scale applied to element
(m, k = n)).  Prints, per row, the (row, block) whose scale each 16-element K group received."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bioengine_worker_amd.ops.fp8 import FP8_DTYPE, linear_fp8_mx

    dev = torch.device("cuda", 0)
    M, K = 16, 128
    xq = torch.ones(M, K).to(FP8_DTYPE).to(dev)
    wq = torch.eye(K).to(FP8_DTYPE).to(dev)  # N = K
    sw = torch.ones(K, device=dev)
    b = torch.arange(K // 32)
    s = (127 + ((torch.arange(M)[:, None] + 3 * b[None, :]) % 8)).to(torch.uint8)
    y = linear_fp8_mx((xq, s.to(dev).contiguous()), wq, sw).float().cpu()
    e = torch.log2(y).round().int()  # applied exponent per (m, k)
    table = {}
    for m in range(M):
        groups = []
        for g in range(K // 16):
            ev = e[m, 16 * g: 16 * g + 16]
            vals = sorted(set(ev.tolist()))
            cands = [(mm, bb) for mm in range(M) for bb in range(K // 32) if (mm + 3 * bb) % 8 in vals]
            groups.append({"k": [16 * g, 16 * g + 15], "exp": vals,
                           "same_row_blocks": [bb for (mm, bb) in cands if mm == m]})
        table[m] = groups
    print(json.dumps({"expected_if_contiguous": "k-group g -> block g // 2 of the same row", "rows": table}))


if __name__ == "__main__":
    main()
