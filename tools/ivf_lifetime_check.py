#!/usr/bin/env python3
"""IVF full-probe recall through VectorIndex.search: as is, with a device sync right after the scan
kernel (operand-lifetime test), and the debug tool's named-operand path."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bioengine_worker_amd.ops import _native  # noqa: E402
from bioengine_worker_amd.search.index import VectorIndex  # noqa: E402

rng = np.random.default_rng(1)
x = rng.normal(size=(30000, 768)).astype(np.float32)
x /= np.linalg.norm(x, axis=1, keepdims=True)
q = x[:24] + 0.05 * rng.normal(size=(24, 768)).astype(np.float32)
idx = VectorIndex(dim=768, device="cuda:0", index_type="ivf", nprobe=8)
idx.add(x)
nl = idx.centroids.shape[0]
flat = np.argsort(-(q @ x.T), axis=1)[:, :10]
rec = lambda I: float(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(I, flat)]))  # noqa: E731
for npb in (256, nl - 1, nl):
    print("as is  nprobe", npb, rec(idx.search(q, 10, nprobe=npb)[1]), flush=True)
orig = _native.call


def synced(name, *a):
    r = orig(name, *a)
    if name == "be_ivf_scan_bf16":
        torch.cuda.synchronize()
    return r


_native.call = synced
for npb in (256, nl - 1, nl):
    print("synced nprobe", npb, rec(idx.search(q, 10, nprobe=npb)[1]), flush=True)
_native.call = orig
S, I = idx.search(q, 10, nprobe=nl)
print("row0 ids", I[0].tolist(), "flat", flat[0].tolist())
print("row0 scores", np.round(S[0], 4).tolist(), "true", np.round(np.sort(q[0] @ x.T)[::-1][:10], 4).tolist())
