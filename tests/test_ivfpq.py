"""IVF-PQ tier (reference FAISS IndexIVFPQ, ``apps/cell-image-search/index_manager.py:67-89``): recall
against exact search, the HIP list-scan kernel against its torch oracle, persistence, and the
VectorIndex tier switch.  FAISS is not installed, so parity with it is unpinned; the oracle is the
exact inner-product ranking."""
import numpy as np
import pytest
import torch

from bioengine_worker_amd.search.index import VectorIndex
from bioengine_worker_amd.search.ivfpq import IVFPQIndex


def _data(n=6000, d=64, nq=20, seed=0):
    g = torch.Generator().manual_seed(seed)
    centers = torch.nn.functional.normalize(torch.randn(40, d, generator=g), dim=1)
    x = centers[torch.randint(0, 40, (n,), generator=g)] + 0.35 * torch.randn(n, d, generator=g)
    x = torch.nn.functional.normalize(x, dim=1)
    q = torch.nn.functional.normalize(x[:nq] + 0.05 * torch.randn(nq, d, generator=g), dim=1)
    return x, q


def _recall(I, gt, k):
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(I, gt)]))


@pytest.mark.unit
def test_ivfpq_recall_and_roundtrip_cpu(tmp_path):
    x, q = _data()
    gt = torch.topk(q @ x.T, 10, dim=1).indices.numpy()
    idx = IVFPQIndex(dim=64, nlist=32, m=16, nprobe=32, device="cpu")
    idx.train(x)
    idx.add(x)
    S, I = idx.search(q, k=10)
    assert I.shape == (20, 10) and (I >= 0).all()
    assert _recall(I, gt, 10) > 0.5 and _recall(I, gt, 1) > 0.9  # 8-bit PQ codes: approximate ranks
    assert np.all(np.diff(S, axis=1) <= 1e-6)  # sorted descending
    # scores approximate the true inner products of the returned ids
    true = (q.numpy()[:, None, :] * x.numpy()[I]).sum(-1)
    assert np.abs(true - S).mean() < 0.05
    idx.save(tmp_path)
    S2, I2 = IVFPQIndex.load(tmp_path, device="cpu").search(q, k=10)
    assert np.array_equal(I, I2)


@pytest.mark.unit
def test_vector_index_ivfpq_tier_cpu(tmp_path):
    x, q = _data(n=3000)
    vi = VectorIndex(dim=64, device="cpu", index_type="ivfpq", pq_m=16, nprobe=40, refine=8)
    vi.add(x)
    assert vi.index_type.startswith("IVFPQ")
    S, I = vi.search(q, k=5)
    assert I.shape == (20, 5) and I[0, 0] == 0  # a query next to x[0] finds it
    # PQ shortlist re-ranked with the exact bf16/fp32 vectors the index keeps (IVFPQ + refine)
    gt = torch.topk(q @ x.T, 5, dim=1).indices.numpy()
    assert _recall(I, gt, 5) > 0.9
    vi.save(tmp_path)
    assert VectorIndex.load(tmp_path, device="cpu").index_type.startswith("IVFPQ")


@pytest.mark.gpu
@pytest.mark.parametrize("m", [96, 192])
def test_ivfpq_scan_kernel_matches_oracle(gpu, m):
    x, q = _data(n=20000, d=768 // 8 * 8, nq=16)
    x, q = torch.nn.functional.pad(x, (0, 768 - x.shape[1])), torch.nn.functional.pad(q, (0, 768 - q.shape[1]))
    idx = IVFPQIndex(dim=768, nlist=64, m=m, nprobe=16, device=gpu)
    idx.train(x.to(gpu))
    idx.add(x.to(gpu))
    S, I = idx.search(q.to(gpu), k=20)
    cpu = IVFPQIndex(dim=768, nlist=64, m=m, nprobe=16, device="cpu")
    cpu.centroids, cpu.codebooks = idx.centroids.cpu(), idx.codebooks.cpu()
    cpu._assign, cpu._raw_codes, cpu.ntotal = idx._assign.cpu(), idx._raw().cpu(), idx.ntotal
    cpu.codes, cpu.ids, cpu.list_off = idx.codes.cpu(), idx.ids.cpu(), idx.list_off.cpu()
    S2, I2 = cpu.search(q, k=20)
    assert np.abs(S - S2).max() < 1e-3
    assert np.mean(I == I2) > 0.95  # ties in fp32 summation order may swap neighbours
    gt = torch.topk(q @ x.T, 20, dim=1).indices.numpy()
    assert _recall(I, gt, 1) > 0.9  # each query's source vector comes back first (dense clusters: top-20 is a coin toss)
