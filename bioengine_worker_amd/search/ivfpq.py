"""IVF-PQ tier of the cell-image-search vector index (reference FAISS ``IndexIVFPQ``, m=96 x 8-bit
codes, nlist in [4096, 65536], nprobe=64: ``apps/cell-image-search/index_manager.py:67-89``; its README
quotes <100 ms per query at 58 M vectors, ``README.md:130-134``).

MI355X design:

* coarse quantizer: spherical k-means on the GPU (bf16 GEMMs), ``nlist`` lists;
* product quantizer on the residuals ``x - c_list``: ``m`` sub-spaces of ``D/m`` dims, 256 centroids
  each, trained with batched k-means (one ``bmm`` per iteration over all sub-spaces);
* codes ``[N, m]`` uint8 stored list-sorted, so each list is one contiguous slab of HBM -- 58 M
  vectors at m=96 are 5.6 GB, scanned for a query only in its ``nprobe`` lists;
* search: per query one ``[m, 256]`` lookup table (``bmm`` of the query's sub-vectors with the
  codebooks, fp16), the HIP kernel ``be_ivfpq_scan`` (one workgroup per (query, list), the table in
  LDS) writes approximate scores for all candidates, then a top-k.  Inner product, so the score is
  ``<q, c_list> + sum_j LUT[j][code_j]``.

Everything has a CPU path (same math in torch) that the GPU kernel is tested against.
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import torch

from ..ops import _native


def _kmeans(x: torch.Tensor, k: int, iters: int, g: torch.Generator, spherical: bool) -> torch.Tensor:
    cent = x[torch.randperm(x.shape[0], generator=g)[:k].to(x.device)].clone()
    for _ in range(iters):
        if spherical:
            from .index import _argmax_ip

            a = _argmax_ip(x, cent)
        else:
            a = torch.cdist(x, cent).argmin(1)
        new = torch.zeros_like(cent).index_add_(0, a, x)
        cnt = torch.bincount(a, minlength=k).to(x.dtype)
        empty = cnt == 0
        new = new / cnt.clamp(min=1)[:, None]
        new[empty] = cent[empty]
        cent = torch.nn.functional.normalize(new, dim=1) if spherical else new
    return cent


def _pq_train(res: torch.Tensor, m: int, iters: int, g: torch.Generator) -> torch.Tensor:
    """Batched k-means (256 centroids) in each of the m sub-spaces: res [S, D] -> codebooks [m, 256, D/m]."""
    S, D = res.shape
    ds = D // m
    x = res.view(S, m, ds).transpose(0, 1).contiguous()  # [m, S, ds]
    init = torch.randperm(S, generator=g)[:256].to(res.device)
    cb = x[:, init].clone()  # [m, 256, ds]
    for _ in range(iters):
        d = (x * x).sum(-1, keepdim=True) - 2 * torch.bmm(x, cb.transpose(1, 2)) + (cb * cb).sum(-1)[:, None, :]
        a = d.argmin(-1)  # [m, S]
        new = torch.zeros_like(cb)
        new.scatter_add_(1, a[..., None].expand(-1, -1, ds), x)
        cnt = torch.zeros(m, 256, device=res.device, dtype=res.dtype).scatter_add_(1, a, torch.ones_like(a, dtype=res.dtype))
        upd = cnt > 0
        cb = torch.where(upd[..., None], new / cnt.clamp(min=1)[..., None], cb)
    return cb


def _pq_encode(res: torch.Tensor, cb: torch.Tensor, chunk: int = 1 << 16) -> torch.Tensor:
    m, _, ds = cb.shape
    out = []
    cbn = (cb * cb).sum(-1)  # [m, 256]
    for i in range(0, res.shape[0], chunk):
        x = res[i:i + chunk].view(-1, m, ds).transpose(0, 1)  # [m, n, ds]
        d = cbn[:, None, :] - 2 * torch.bmm(x, cb.transpose(1, 2))
        out.append(d.argmin(-1).transpose(0, 1).to(torch.uint8))
    return torch.cat(out).contiguous()


class IVFPQIndex:
    """Approximate inner-product index; vectors should be L2-normalised (cosine)."""

    def __init__(self, dim: int = 768, nlist: int = 4096, m: int = 96, nprobe: int = 64, device=None):
        if dim % m or m % 16:
            raise ValueError("dim must be divisible by m, and m a multiple of 16")
        self.dim, self.nlist, self.m, self.nprobe = dim, nlist, m, nprobe
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.centroids: torch.Tensor | None = None  # [nlist, D] fp32
        self.codebooks: torch.Tensor | None = None  # [m, 256, D/m] fp32
        self.codes = torch.empty(0, m, dtype=torch.uint8, device=self.device)  # list-sorted
        self.ids = torch.empty(0, dtype=torch.int64, device=self.device)  # original id per sorted row
        self.list_off = torch.zeros(nlist + 1, dtype=torch.int64, device=self.device)
        self._assign = torch.empty(0, dtype=torch.int32, device=self.device)
        self._raw_codes = torch.empty(0, m, dtype=torch.uint8, device=self.device)
        self.ntotal = 0

    @property
    def index_type(self) -> str:
        return f"IVFPQ-GPU(nlist={self.nlist}, m={self.m}, nbits=8)"

    # ------------------------------------------------------------------ build
    def train(self, x, iters: int = 10, pq_iters: int = 12, seed: int = 0, max_sample: int = 262_144,
              pq_sample: int = 65_536) -> None:
        x = torch.as_tensor(x).to(self.device, torch.float32)
        g = torch.Generator().manual_seed(seed)
        n = x.shape[0]
        sample = x[torch.randperm(n, generator=g)[: min(n, max(max_sample, 39 * self.nlist))].to(self.device)]
        self.centroids = _kmeans(sample, min(self.nlist, sample.shape[0]), iters, g, spherical=True)
        self.nlist = self.centroids.shape[0]
        self.list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        ps = sample[:pq_sample]  # PQ codebooks: 256 centroids per sub-space need far fewer points
        from .index import _argmax_ip

        a = _argmax_ip(ps, self.centroids)
        self.codebooks = _pq_train(ps - self.centroids[a], self.m, pq_iters, g)

    def add(self, x, chunk: int = 1 << 18) -> None:
        assert self.centroids is not None, "train() first"
        x = torch.as_tensor(x)
        assigns, codes = [], []
        for i in range(0, x.shape[0], chunk):
            xc = x[i:i + chunk].to(self.device, torch.float32)
            from .index import _argmax_ip

            a = _argmax_ip(xc, self.centroids)
            codes.append(_pq_encode(xc - self.centroids[a], self.codebooks))
            assigns.append(a.int())
        self._assign = torch.cat([self._assign] + assigns)
        raw = torch.cat([self._raw()] + codes)
        self.ntotal = int(self._assign.shape[0])
        order = torch.argsort(self._assign, stable=True)
        self.codes = raw[order].contiguous()
        self.ids = order
        # id-order codes are not kept: the list-sorted copy + ids reconstruct them (_raw), so the GPU
        # holds m + 12 bytes per vector (204 B at m = 192: 11.8 GB at 58 M)
        self._raw_codes = None
        del raw
        counts = torch.bincount(self._assign.long(), minlength=self.nlist)
        self.list_off = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])

    def _raw(self) -> torch.Tensor:
        """Codes in id order [N, m]."""
        if self._raw_codes is not None:
            return self._raw_codes
        raw = torch.empty_like(self.codes)
        raw[self.ids] = self.codes
        return raw

    def gpu_bytes(self) -> int:
        t = [self.codes, self.ids, self._assign, self.centroids, self.codebooks, self.list_off]
        return int(sum(x.numel() * x.element_size() for x in t if x is not None))

    # ------------------------------------------------------------------ search
    def _lut(self, q: torch.Tensor) -> torch.Tensor:
        """[Q, m, 256]: <q_j, codebook_j[k]>."""
        Q = q.shape[0]
        ds = self.dim // self.m
        qs = q.view(Q, self.m, ds).transpose(0, 1)  # [m, Q, ds]
        return torch.bmm(qs, self.codebooks.transpose(1, 2)).transpose(0, 1).contiguous()  # [m,Q,256] -> [Q,m,256]

    @torch.no_grad()
    def search(self, q, k: int = 20, nprobe: int | None = None):
        """q [Q, D] -> (scores [Q, k] fp32 numpy, ids [Q, k] int64 numpy; -1 = empty slot)."""
        q = torch.as_tensor(np.asarray(q, np.float32) if not torch.is_tensor(q) else q).to(self.device, torch.float32)
        if q.dim() == 1:
            q = q[None]
        Q = q.shape[0]
        nprobe = min(nprobe or self.nprobe, self.nlist)
        cs = q @ self.centroids.T
        base, probes = torch.topk(cs, nprobe, dim=1)
        sizes = (self.list_off[1:] - self.list_off[:-1])[probes]  # [Q, nprobe]
        cand_off = torch.cumsum(sizes, 1) - sizes
        tot = sizes.sum(1)
        stride = int(tot.max()) if Q else 0
        S = np.full((Q, k), -np.inf, np.float32)
        I = np.full((Q, k), -1, np.int64)
        if stride == 0:
            return S, I
        lut = self._lut(q)
        out = torch.full((Q, stride), -float("inf"), dtype=torch.float32, device=self.device)
        if self.device.type == "cuda":
            _native.call("be_ivfpq_scan", _native.ptr(lut.half().contiguous()), _native.ptr(base.contiguous()),
                         _native.ptr(probes.int().contiguous()), _native.ptr(self.list_off), _native.ptr(cand_off.contiguous()),
                         _native.ptr(self.codes), Q, nprobe, self.m, stride, _native.ptr(out), _native.stream(self.device))
        else:
            self._scan_reference(lut, base, probes, cand_off, out)
        kk = min(k, stride)
        ts, ti = torch.topk(out, kk, dim=1)
        # candidate slot -> list-sorted row -> original id
        rows = self._slot_rows(probes, cand_off, sizes, ti)
        ids = torch.where(torch.isfinite(ts), self.ids[rows.clamp(min=0)], torch.full_like(rows, -1))
        S[:, :kk] = ts.cpu().numpy()
        I[:, :kk] = ids.cpu().numpy()
        return S, I

    def _slot_rows(self, probes, cand_off, sizes, slots):
        """Candidate-row slot index -> list-sorted code row."""
        # which probed list holds the slot: last p with cand_off[p] <= slot
        p = torch.searchsorted(cand_off.contiguous(), slots.contiguous(), right=True) - 1
        p = p.clamp(min=0)
        lists = torch.gather(probes, 1, p)
        within = slots - torch.gather(cand_off, 1, p)
        return self.list_off[lists] + within

    def _scan_reference(self, lut, base, probes, cand_off, out):
        """torch oracle of be_ivfpq_scan (same fp16 table)."""
        lh = lut.half().float()
        for qi in range(probes.shape[0]):
            for pi in range(probes.shape[1]):
                l = int(probes[qi, pi])
                a, b = int(self.list_off[l]), int(self.list_off[l + 1])
                if a == b:
                    continue
                c = self.codes[a:b].long()  # [n, m]
                s = lh[qi].gather(1, c.T).sum(0) + base[qi, pi]
                o = int(cand_off[qi, pi])
                out[qi, o:o + (b - a)] = s

    # ------------------------------------------------------------------ persistence
    def save(self, out_dir) -> dict:
        out = Path(out_dir)
        out.mkdir(parents=True, exist_ok=True)
        np.save(out / "ivfpq_centroids.npy", self.centroids.cpu().numpy())
        np.save(out / "ivfpq_codebooks.npy", self.codebooks.cpu().numpy())
        np.save(out / "ivfpq_codes.npy", self._raw().cpu().numpy())
        np.save(out / "ivfpq_assign.npy", self._assign.cpu().numpy())
        info = {"n_cells": self.ntotal, "embed_dim": self.dim, "index_type": self.index_type, "nprobe": self.nprobe,
                "index_size_mb": round(self.codes.numel() / 2 ** 20, 3)}
        (out / "ivfpq_info.json").write_text(json.dumps(info, indent=2))
        return info

    @classmethod
    def load(cls, out_dir, device=None) -> "IVFPQIndex":
        out = Path(out_dir)
        info = json.loads((out / "ivfpq_info.json").read_text())
        cent = np.load(out / "ivfpq_centroids.npy")
        cb = np.load(out / "ivfpq_codebooks.npy")
        idx = cls(dim=info["embed_dim"], nlist=cent.shape[0], m=cb.shape[0], nprobe=info.get("nprobe", 64), device=device)
        idx.centroids = torch.from_numpy(cent).to(idx.device)
        idx.codebooks = torch.from_numpy(cb).to(idx.device)
        codes = torch.from_numpy(np.load(out / "ivfpq_codes.npy")).to(idx.device)
        assign = torch.from_numpy(np.load(out / "ivfpq_assign.npy")).to(idx.device)
        idx._assign = assign
        idx.ntotal = int(assign.shape[0])
        order = torch.argsort(assign, stable=True)
        idx.codes, idx.ids = codes[order].contiguous(), order
        idx._raw_codes = None
        counts = torch.bincount(assign.long(), minlength=idx.nlist)
        idx.list_off = torch.cat([counts.new_zeros(1), torch.cumsum(counts, 0)])
        return idx


def default_nlist(n: int) -> int:
    """Reference range nlist in [4096, 65536] around 4*sqrt(N) (FAISS guideline)."""
    return int(min(65536, max(4096, 4 * math.sqrt(max(n, 1)))))
