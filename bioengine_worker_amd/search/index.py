"""GPU vector index for L2-normalised embeddings (inner product = cosine).

Replaces the reference's FAISS indexes (apps/cell-image-search/index_manager.py:36-182,
SURVEY.md K20) with an HBM-resident design: MI355X holds 288 GB, i.e. ~180 M 768-d bf16 vectors,
so exact search is one bf16 GEMM (hipBLASLt) per query batch plus a top-k, streamed over
fixed-size chunks.  Past ``ivf_threshold`` vectors an IVF layer (spherical k-means on the GPU,
``nlist ~ 4 sqrt(N)``, ``nprobe = 64`` as in the reference) restricts each query to its closest
lists, whose list-sorted bf16 slabs are scored EXACTLY by the HIP scan kernel
(``csrc/kernels/ivf_scan.hip``) -- the reference needs 8-bit PQ codes at this size because it is
CPU/DRAM bound; on one 288 GB GPU the full vectors fit, so recall is limited only by probing.  The
compressed IVF-PQ tier (``search/ivfpq.py``) is kept for collections that do not fit:
:meth:`VectorIndex.compress` keeps only the PQ codes on the GPU (m=192: 192 B per vector, 11 GB at
58 M) and moves the full vectors to HOST memory, where the PQ shortlist (``refine * k``
candidates) is gathered and re-scored exactly on the GPU -- FAISS ``IndexRefineFlat`` with the
refine store off the device.  Storage is plain ``.npy`` + JSON (no pickles).

Layout at ``<workspace>/cell_search/``: ``vectors.npy`` (fp16 [N, D]), ``index_info.json``,
``ivf_centroids.npy`` / ``ivf_assign.npy`` (IVF only), ``metadata.parquet``, ``thumbnails.npy``.
"""
from __future__ import annotations

import json
import math
import time
from pathlib import Path

import numpy as np
import torch

CHUNK = 1 << 20  # database rows per GEMM chunk


def _scores(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """q [Q, D] x v [n, D] -> fp32 [Q, n].  bf16 GEMMs keep fp32 outputs (``mm.dtype``): bf16-rounded
    scores (8 mantissa bits, ~0.004 near 1.0) tie near-duplicate neighbours and scramble the top-k."""
    if q.is_cuda and q.dtype == torch.bfloat16:
        return torch.mm(q, v.T, out_dtype=torch.float32)
    return (q @ v.T).float()


def _argmax_ip(x: torch.Tensor, cent: torch.Tensor, budget: int = 1 << 30) -> torch.Tensor:
    """Nearest centroid by inner product, in row chunks sized so the [rows, nlist] score block stays
    under ``budget`` elements (at 58 M x 30 k lists an unchunked product would be ~7 TB)."""
    cent = cent.to(x.dtype)
    rows = max(1, min(x.shape[0], budget // max(1, cent.shape[0])))
    return torch.cat([(x[i:i + rows] @ cent.T).argmax(1) for i in range(0, x.shape[0], rows)])


class VectorIndex:
    """Tiers (reference FlatIP / IVFFlat / IVFPQ): ``index_type="auto"`` keeps exact bf16 search up
    to ``ivf_threshold`` vectors, IVF-Flat above it and IVF-PQ (``search/ivfpq.py``, m=96 x 8 bit)
    from ``ivfpq_threshold``; ``"flat"`` / ``"ivf"`` / ``"ivfpq"`` force a tier."""

    def __init__(self, dim: int = 768, device=None, ivf_threshold: int = 5_000_000, nprobe: int = 64,
                 index_type: str = "auto", ivfpq_threshold: int = 50_000_000, pq_m: int = 96, refine: int = 4):
        self.lvecs: torch.Tensor | None = None
        self.dim = dim
        self.refine = refine  # IVF-PQ: re-rank refine*k PQ candidates with the stored vectors (0 = off)
        self.kind = index_type
        self.ivfpq_threshold = ivfpq_threshold
        self.pq_m = pq_m
        self.pq = None
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.vecs = torch.empty(0, dim, dtype=self.dtype, device=self.device)
        self.ivf_threshold = ivf_threshold
        self.nprobe = nprobe
        self.centroids: torch.Tensor | None = None
        self.assign: torch.Tensor | None = None
        self.lists: list[torch.Tensor] | None = None
        self.host_refine = False  # compressed tier: self.vecs lives in host memory (refine store only)

    # ------------------------------------------------------------------ build
    @property
    def ntotal(self) -> int:
        return int(self.vecs.shape[0])

    @property
    def index_type(self) -> str:
        if self.pq is not None:
            return self.pq.index_type
        return f"IVFFlat-GPU(nlist={self.centroids.shape[0]})" if self.centroids is not None else "FlatIP-GPU"

    def add(self, x) -> None:
        x = torch.as_tensor(np.asarray(x, np.float32) if not torch.is_tensor(x) else x).to(self.device, self.dtype)
        assert x.dim() == 2 and x.shape[1] == self.dim
        self.vecs = torch.cat([self.vecs, x.to(self.vecs.device)], 0)
        if self.pq is not None:
            self.pq.add(x.float())
        elif self.kind == "ivfpq" or (self.kind == "auto" and self.ntotal >= self.ivfpq_threshold
                                       and not self._fits_hbm(self.ntotal)):
            self.train_ivfpq()
        elif self.centroids is not None:
            self._assign_new(x, self.ntotal - x.shape[0])
        elif self.kind == "ivf" or (self.kind == "auto" and self.ntotal >= self.ivf_threshold):
            self.train_ivf()

    def _fits_hbm(self, n: int) -> bool:
        """The exact-scan IVF tier keeps the vectors twice (id order + list-sorted): use it while
        that fits in a third of this GPU's HBM (58 M x 768 bf16 x 2 = 178 GB of 288 GB: yes)."""
        if self.device.type != "cuda":
            return False
        total = torch.cuda.get_device_properties(self.device).total_memory
        return 2 * n * self.dim * 2 <= 0.66 * total

    def train_ivfpq(self, nlist: int | None = None) -> None:
        from .ivfpq import IVFPQIndex, default_nlist

        n = self.ntotal
        nl = nlist or min(default_nlist(n), max(1, n // 39))
        pq = IVFPQIndex(self.dim, nl, self.pq_m, self.nprobe, self.device)
        g = torch.Generator(device="cpu").manual_seed(0)
        sample = self.vecs[torch.randperm(n, generator=g)[: min(n, max(262_144, 39 * nl))].to(self.vecs.device)]
        pq.train(sample.float())
        for i in range(0, n, 1 << 22):  # encode in chunks: no fp32 copy of the whole collection
            pq.add(self.vecs[i:i + (1 << 22)].float())
        self.pq = pq
        self.centroids = None

    def compress(self, pq_m: int = 192, refine: int = 50, nlist: int | None = None) -> dict:
        """Switch to the compressed tier: IVF-PQ codes (``pq_m`` bytes per vector) on the GPU, the full
        vectors in host memory as the exact re-rank store.  Search returns the top-k of the
        ``refine * k`` PQ candidates re-scored exactly.  Returns the GPU / host footprint (bytes)."""
        self.pq_m, self.refine = pq_m, refine
        self.lvecs = None
        self.train_ivfpq(nlist)
        self.vecs = self.vecs.cpu()  # bf16 on the host: ~1.5 KB per vector, gathered per query
        self.host_refine = True
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        return {"gpu_bytes": self.pq.gpu_bytes(), "host_bytes": int(self.vecs.numel() * self.vecs.element_size())}

    def _refine_rows(self, c: torch.Tensor) -> torch.Tensor:
        """[Q, R] candidate ids (>= 0) -> their stored vectors [Q, R, D] on the index device."""
        if not self.host_refine:
            return self.vecs[c]
        rows = self.vecs.index_select(0, c.reshape(-1).cpu())  # host gather (multi-threaded)
        return rows.to(self.device, non_blocking=False).view(*c.shape, self.dim)

    def train_ivf(self, nlist: int | None = None, iters: int = 10, seed: int = 0) -> None:
        n = self.ntotal
        # ~4 sqrt(N) lists (the FAISS guideline the reference's IVF-PQ tier follows): at 58 M that is
        # ~30 k lists of ~1.9 k vectors, so nprobe 64 scans ~120 k exact candidates per query
        nlist = nlist or int(min(65536, max(64, 4 * math.sqrt(n))))
        g = torch.Generator(device="cpu").manual_seed(seed)
        # 64 points per list (FAISS trains IVF on 39-256 per list); scores in the storage dtype
        sample = self.vecs[torch.randperm(n, generator=g)[: min(n, 64 * nlist)].to(self.device)]
        samplef = sample.float()
        cent = samplef[torch.randperm(sample.shape[0], generator=g)[:nlist].to(self.device)].clone()
        for _ in range(iters):  # spherical k-means
            a = _argmax_ip(sample, cent)
            new = torch.zeros_like(cent).index_add_(0, a, samplef)
            cnt = torch.bincount(a, minlength=nlist)
            empty = cnt == 0
            new[empty] = cent[empty]
            cent = torch.nn.functional.normalize(new, dim=1)
        self.centroids = cent.to(self.dtype)
        self.assign = torch.empty(0, dtype=torch.int32, device=self.device)
        self._assign_new(self.vecs, 0)

    def _assign_new(self, x: torch.Tensor, base: int) -> None:
        a = _argmax_ip(x, self.centroids).int()
        self.assign = torch.cat([self.assign, a])
        order = torch.argsort(self.assign, stable=True)
        counts = torch.bincount(self.assign.long(), minlength=self.centroids.shape[0])
        self.sorted_ids = order  # vector ids grouped by list
        self.list_off = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])
        self.lists = None
        # list-sorted copy of the vectors: every IVF list is one contiguous HBM slab that the exact
        # scan kernel streams (be_ivf_scan_bf16); built chunk by chunk to bound the temporary
        # (be_ivf_scan_bf16 is instantiated for dim/128 in {1,2,3,4,6,8}; other dims use the bmm path)
        if self.device.type == "cuda" and self.dim % 128 == 0 and self.dim // 128 in (1, 2, 3, 4, 6, 8):
            lv = torch.empty_like(self.vecs)
            for i in range(0, order.numel(), CHUNK):
                lv[i:i + CHUNK] = self.vecs[order[i:i + CHUNK]]
            self.lvecs = lv
        else:
            self.lvecs = None

    # ------------------------------------------------------------------ search
    @torch.no_grad()
    def search(self, q, k: int = 20, nprobe: int | None = None):
        """q [Q, D] -> (scores [Q, k] fp32 numpy, ids [Q, k] int64 numpy; -1 = empty slot).
        ``nprobe`` overrides the IVF probe count for this call."""
        q = torch.as_tensor(np.asarray(q, np.float32) if not torch.is_tensor(q) else q).to(self.device, self.dtype)
        if q.dim() == 1:
            q = q[None]
        Q = q.shape[0]
        k_eff = min(k, self.ntotal)
        if k_eff == 0:
            return np.full((Q, k), -np.inf, np.float32), np.full((Q, k), -1, np.int64)
        if self.pq is not None:
            if not self.refine or self.vecs.shape[0] != self.ntotal:
                return self.pq.search(q.float(), k)
            # IVF-PQ shortlist of refine*k, re-scored exactly with the stored vectors (IVFPQ+R)
            _, cand = self.pq.search(q.float(), self.refine * k)
            c = torch.from_numpy(cand).to(self.device)
            ok = c >= 0
            s = torch.einsum("qd,qkd->qk", q.float(), self._refine_rows(c.clamp(min=0)).float())
            s = torch.where(ok, s, torch.full_like(s, -float("inf")))
            ts, ti = torch.topk(s, min(k, s.shape[1]), dim=1)
            ids = torch.where(torch.isfinite(ts), torch.gather(c, 1, ti), torch.full_like(ti, -1))
            S = np.full((Q, k), -np.inf, np.float32)
            I = np.full((Q, k), -1, np.int64)
            S[:, : ts.shape[1]] = ts.cpu().numpy()
            I[:, : ids.shape[1]] = ids.cpu().numpy()
            return S, I
        if self.centroids is None:
            best_s = torch.full((Q, 0), -float("inf"), device=self.device)
            best_i = torch.empty(Q, 0, dtype=torch.long, device=self.device)
            for i in range(0, self.ntotal, CHUNK):
                s = _scores(q, self.vecs[i:i + CHUNK])
                ts, ti = torch.topk(s, min(k_eff, s.shape[1]), dim=1)
                best_s = torch.cat([best_s, ts], 1)
                best_i = torch.cat([best_i, ti + i], 1)
                best_s, j = torch.topk(best_s, min(k_eff, best_s.shape[1]), dim=1)
                best_i = torch.gather(best_i, 1, j)
        else:
            best_s, best_i = self._search_ivf(q, k_eff, nprobe=nprobe)
        S = np.full((Q, k), -np.inf, np.float32)
        I = np.full((Q, k), -1, np.int64)
        S[:, : best_s.shape[1]] = best_s.cpu().numpy()
        I[:, : best_i.shape[1]] = best_i.cpu().numpy()
        return S, I

    def _search_ivf(self, q: torch.Tensor, k: int, q_chunk: int = 8, nprobe: int | None = None):
        """Batched IVF-Flat: every query's probed lists become one padded candidate row (list-sorted
        vector ids, located through the list offsets).  GPU: the HIP scan kernel scores every
        candidate exactly from the list-sorted bf16 slabs, then one top-k; CPU: one batched GEMM
        per query chunk.  No per-query Python loop either way."""
        nl = self.centroids.shape[0]
        npb = min(nprobe or self.nprobe, nl)
        if npb == nl:  # every list: no ranking needed (the candidate order does not matter)
            probes = torch.arange(nl, device=q.device).expand(q.shape[0], nl).contiguous()
        else:
            probes = torch.topk((q @ self.centroids.T).float(), npb, dim=1).indices
        sizes = (self.list_off[1:] - self.list_off[:-1])[probes]  # [Q, nprobe]
        cand_off = torch.cumsum(sizes, 1) - sizes
        stride = int(sizes.sum(1).max())
        Q = q.shape[0]
        best_s = torch.full((Q, k), -float("inf"), device=self.device)
        best_i = torch.full((Q, k), -1, dtype=torch.long, device=self.device)
        if stride == 0:
            return best_s, best_i
        if getattr(self, "lvecs", None) is not None and self.lvecs.shape[0] == self.ntotal:
            from ..ops import _native

            out = torch.full((Q, stride), -float("inf"), dtype=torch.float32, device=self.device)
            _native.call("be_ivf_scan_bf16", _native.ptr(q.float().contiguous()), _native.ptr(probes.int().contiguous()),
                         _native.ptr(self.list_off), _native.ptr(cand_off.contiguous()), _native.ptr(self.lvecs), Q,
                         probes.shape[1], self.dim, stride, _native.ptr(out), _native.stream(self.device))
            ts, ti = torch.topk(out, min(k, stride), dim=1)
            p = (torch.searchsorted(cand_off.contiguous(), ti.contiguous(), right=True) - 1).clamp(min=0)
            rows = self.list_off[torch.gather(probes, 1, p)] + (ti - torch.gather(cand_off, 1, p))
            ids = self.sorted_ids[rows.clamp(0, self.ntotal - 1)]
            best_s[:, : ts.shape[1]] = ts
            best_i[:, : ts.shape[1]] = torch.where(torch.isfinite(ts), ids, torch.full_like(ids, -1))
            return best_s, best_i
        slots = torch.arange(stride, device=self.device)
        for a in range(0, Q, q_chunk):
            b = min(Q, a + q_chunk)
            sl = slots.expand(b - a, stride).contiguous()
            p = (torch.searchsorted(cand_off[a:b].contiguous(), sl, right=True) - 1).clamp(min=0)
            lists = torch.gather(probes[a:b], 1, p)
            within = sl - torch.gather(cand_off[a:b], 1, p)
            valid = within < torch.gather(sizes[a:b], 1, p)
            rows = (self.list_off[lists] + within).clamp(max=self.sorted_ids.numel() - 1)
            ids = self.sorted_ids[rows]
            sc = torch.bmm(self.vecs[ids], q[a:b, :, None]).squeeze(-1).float()
            sc = torch.where(valid, sc, torch.full_like(sc, -float("inf")))
            ts, ti = torch.topk(sc, min(k, stride), dim=1)
            best_s[a:b, : ts.shape[1]] = ts
            best_i[a:b, : ts.shape[1]] = torch.where(torch.isfinite(ts), torch.gather(ids, 1, ti), torch.full_like(ti, -1))
        return best_s, best_i

    def reconstruct_batch(self, ids) -> np.ndarray:
        return self.vecs[torch.as_tensor(np.asarray(ids), device=self.vecs.device)].float().cpu().numpy()

    # ------------------------------------------------------------------ persistence
    def save(self, out_dir) -> dict:
        out = Path(out_dir)
        out.mkdir(parents=True, exist_ok=True)
        t0 = time.time()
        np.save(out / "vectors.npy", self.vecs.float().cpu().numpy().astype(np.float16))
        if self.pq is not None:
            self.pq.save(out)
        else:
            (out / "ivfpq_info.json").unlink(missing_ok=True)
        if self.centroids is not None:
            np.save(out / "ivf_centroids.npy", self.centroids.float().cpu().numpy())
        else:
            (out / "ivf_centroids.npy").unlink(missing_ok=True)
        info = {"n_cells": self.ntotal, "embed_dim": self.dim, "index_type": self.index_type,
                "host_refine": self.host_refine, "refine": self.refine,
                "index_size_mb": round((out / "vectors.npy").stat().st_size / 2 ** 20, 3),
                "build_seconds": round(time.time() - t0, 3),
                "build_time_iso": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        (out / "index_info.json").write_text(json.dumps(info, indent=2))
        return info

    @classmethod
    def load(cls, out_dir, device=None) -> "VectorIndex":
        out = Path(out_dir)
        p = out / "vectors.npy"
        if not p.exists():
            raise FileNotFoundError(f"No index at {p}")
        v = np.load(p)  # allow_pickle=False
        idx = cls(dim=v.shape[1], device=device)
        ii = out / "index_info.json"
        info = json.loads(ii.read_text()) if ii.exists() else {}
        host = bool(info.get("host_refine")) and (out / "ivfpq_info.json").exists()
        idx.vecs = torch.from_numpy(v.astype(np.float32)).to("cpu" if host else idx.device, idx.dtype)
        if (out / "ivfpq_info.json").exists():
            from .ivfpq import IVFPQIndex

            idx.pq = IVFPQIndex.load(out, device=idx.device)
            idx.host_refine = host
            idx.refine = int(info.get("refine", idx.refine))
            idx.pq_m = idx.pq.m
            return idx
        c = out / "ivf_centroids.npy"
        if c.exists():
            idx.centroids = torch.from_numpy(np.load(c)).to(idx.device, idx.dtype)
            idx.assign = torch.empty(0, dtype=torch.int32, device=idx.device)
            idx._assign_new(idx.vecs, 0)
        return idx
