#!/usr/bin/env python3
"""Are the IVF probe lists of tools/ivf_scan_debug.py's index unique per query on the GPU
(torch.topk over all centroids), and does torch.sort agree?"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bioengine_worker_amd.search.index import VectorIndex  # noqa: E402

rng = np.random.default_rng(1)
x = rng.normal(size=(30000, 768)).astype(np.float32)
x /= np.linalg.norm(x, axis=1, keepdims=True)
q = x[:24] + 0.05 * rng.normal(size=(24, 768)).astype(np.float32)
idx = VectorIndex(dim=768, device="cuda:0", index_type="ivf", nprobe=8)
idx.add(x)
nl = idx.centroids.shape[0]
qt = torch.from_numpy(q).cuda().bfloat16()
sc = (qt @ idx.centroids.T).float()
for k in (8, 256, 512, 600, nl):
    pt = torch.topk(sc, k, dim=1).indices
    ps = torch.sort(sc, dim=1, descending=True).indices[:, :k]
    pc = torch.topk(sc.cpu(), k, dim=1).indices
    uniq = min(len(set(r.tolist())) for r in pt.cpu())
    print("k", k, "min unique per row", uniq, "topk==cpu topk sets", all(set(a.tolist()) == set(b.tolist()) for a, b in zip(pt.cpu(), pc)),
          "sort==cpu sets", all(set(a.tolist()) == set(b.tolist()) for a, b in zip(ps.cpu(), pc)), flush=True)
print("vecs == lvecs[argsort(sorted_ids)]:", bool(torch.equal(idx.lvecs[torch.argsort(idx.sorted_ids)], idx.vecs)))
