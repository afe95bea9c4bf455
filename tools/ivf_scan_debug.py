#!/usr/bin/env python3
"""Debug of the full-probe IVF exact-scan path (tests/test_search_gpu.py::test_ivf_exact_scan_...):
the scan kernel's candidate scores against a torch recomputation over the same candidate layout."""
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
for npb in (8, 64, 256, nl):
    S, I = idx.search(q, 10, nprobe=npb)
    rec = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(I, flat)])
    print("nprobe", npb, "recall vs flat", rec, flush=True)
qt = torch.from_numpy(q).cuda().bfloat16()
probes = torch.topk((qt @ idx.centroids.T).float(), nl, dim=1).indices
sizes = (idx.list_off[1:] - idx.list_off[:-1])[probes]
cand_off = torch.cumsum(sizes, 1) - sizes
stride = int(sizes.sum(1).max())
out = torch.full((24, stride), -float("inf"), device="cuda")
qf = qt.float().contiguous()
pi = probes.int().contiguous()
co = cand_off.contiguous()
_native.call("be_ivf_scan_bf16", _native.ptr(qf), _native.ptr(pi), _native.ptr(idx.list_off), _native.ptr(co),
             _native.ptr(idx.lvecs), 24, nl, 768, stride, _native.ptr(out), _native.stream(torch.device("cuda:0")))
torch.cuda.synchronize()
# reference: candidate slot j of query i = row list_off[probe] + (j - cand_off[probe]) of lvecs
ref = torch.full_like(out, -float("inf"))
for i in range(24):
    rows = torch.cat([torch.arange(int(idx.list_off[l]), int(idx.list_off[l + 1]), device="cuda") for l in probes[i].tolist()])
    ref[i, : rows.numel()] = idx.lvecs[rows].float() @ qf[i]
d = (out - ref).abs()
d[torch.isinf(ref) & torch.isinf(out)] = 0
print("max |scan - ref|", float(d.max()), "bad slots", int((d > 1e-2).sum()), "of", out.numel(), flush=True)
print("dtype list_off", idx.list_off.dtype, "cand_off", cand_off.dtype, "probes", probes.dtype, "stride", stride)
# post-processing of the scan output on the GPU vs the same tensors on the CPU
def post(out, probes, cand_off, list_off, sorted_ids, ntotal):
    ts, ti = torch.topk(out, 10, dim=1)
    p = (torch.searchsorted(cand_off.contiguous(), ti.contiguous(), right=True) - 1).clamp(min=0)
    rows = list_off[torch.gather(probes, 1, p)] + (ti - torch.gather(cand_off, 1, p))
    ids = sorted_ids[rows.clamp(0, ntotal - 1)]
    return ts, ti, p, rows, ids


g = post(out, probes, cand_off, idx.list_off, idx.sorted_ids, idx.ntotal)
c = post(out.cpu(), probes.cpu(), cand_off.cpu(), idx.list_off.cpu(), idx.sorted_ids.cpu(), idx.ntotal)
for name, a, b in zip(("ts", "ti", "p", "rows", "ids"), g, c):
    a = a.cpu()
    print(name, "mismatches", int((a != b).sum()), "of", a.numel(), flush=True)
print("empty lists", int(((idx.list_off[1:] - idx.list_off[:-1]) == 0).sum()), "of", nl)
ssg = torch.searchsorted(cand_off.contiguous(), g[1].contiguous(), right=True)
ssc = torch.searchsorted(cand_off.cpu().contiguous(), g[1].cpu().contiguous(), right=True)
print("searchsorted gpu vs cpu mismatches", int((ssg.cpu() != ssc).sum()))
i = int(torch.nonzero((ssg.cpu() != ssc).any(1))[0]) if (ssg.cpu() != ssc).any() else None
if i is not None:
    print("row", i, "ti", g[1][i].tolist(), "gpu", ssg[i].tolist(), "cpu", ssc[i].tolist())
