"""3-D EM volumes: slice-wise tiled inference, 3-D instances, and z-slab sharding across GPUs.

The reference analyses 2-D images only (tiles shipped to a model service); SURVEY.md §2.7 makes
spatial tiling the "context parallel" axis of the rebuild and §2.6 C12(b) names the RCCL
all-gather of stitched slabs.  A 2048^3 uint8 volume (8.6 GB) fits one MI355X's 288 GB many times,
but its probability map and labels are computed fastest with every GPU of the node working on
its own z-slab:

* each rank takes a contiguous z-slab (balanced split), runs slice-wise tiled inference on it and
  thresholds it;
* each rank labels its slab with the 6-connected HIP union-find CCL (slab < 2^31 voxels);
* ranks exchange their first/last label slices (one all-gather of 2 x Y x X int32 per rank),
  rank 0 unions labels that touch across slab faces and broadcasts the global relabel table;
* labels become globally consistent; per-instance voxel counts and centroids are reduced with one
  all-reduce.  The full label volume is optionally all-gathered (``gather_labels``).

Works with any ``torch.distributed`` process group (``nccl`` = RCCL over xGMI on the GPU node,
``gloo`` for CPU tests).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ..ops import _native
from . import mito


def slab_bounds(Z: int, rank: int, world: int) -> tuple[int, int]:
    base, rem = divmod(Z, world)
    z0 = rank * base + min(rank, rem)
    return z0, z0 + base + (1 if rank < rem else 0)


def ccl3d(mask: torch.Tensor) -> torch.Tensor:
    """6-connected components; int32 root index per voxel (-1 background)."""
    if not mask.is_cuda:
        from scipy import ndimage

        lab, _ = ndimage.label(mask.cpu().numpy(), structure=ndimage.generate_binary_structure(3, 1))
        lab = lab.astype(np.int64)
        # root = first voxel (raster order) of each component, like the GPU kernel
        flat = lab.ravel()
        first = np.full(flat.max() + 1, -1, np.int64)
        idx = np.nonzero(flat)[0]
        order = np.unique(flat[idx], return_index=True)
        first[order[0]] = idx[order[1]]
        out = np.where(flat > 0, first[flat], -1).reshape(lab.shape).astype(np.int32)
        return torch.from_numpy(out)
    D, H, W = mask.shape
    m = mask.to(torch.uint8).contiguous()
    lab = torch.empty(D, H, W, dtype=torch.int32, device=mask.device)
    _native.call("be_ccl3d", _native.ptr(m), D, H, W, _native.ptr(lab), _native.stream(mask.device))
    return lab


def slice_probabilities(vol: torch.Tensor, predict, tile: int = 512, overlap: int = 64, batch: int = 8) -> torch.Tensor:
    """[Z, Y, X] normalised volume -> foreground probability [Z, Y, X] (slice-wise 2-D model)."""
    out = torch.empty(vol.shape, dtype=torch.float32, device=vol.device)
    Z, Y, X = vol.shape
    for z in range(Z):
        if Y <= tile and X <= tile:
            out[z] = predict(vol[z][None, None])[0, 0]
        else:
            out[z] = mito.infer_tiled(vol[z], predict, tile, overlap, batch)[0]
    return out


def _union_find_pairs(pairs: np.ndarray, n: int) -> np.ndarray:
    parent = np.arange(n)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a

    for a, b in pairs:
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    return np.array([find(i) for i in range(n)])


def label_sharded(mask_slab: torch.Tensor, group=None) -> tuple[torch.Tensor, int]:
    """Globally consistent instance labels (1..N) for z-slab ``mask_slab`` of this rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    roots = ccl3d(mask_slab).to(mask_slab.device)
    local, n_local = mito.compact_labels(roots)  # 1..n_local in slab raster order
    if world == 1:
        return local, n_local
    dev = mask_slab.device
    counts = torch.tensor([n_local], dtype=torch.int64, device=dev)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts, group=group)
    offs = np.concatenate([[0], np.cumsum([int(c) for c in all_counts])])
    glob = torch.where(local > 0, local + int(offs[rank]), local)
    Y, X = mask_slab.shape[1:]
    faces = torch.stack([glob[0], glob[-1]]).to(torch.int64)
    gathered = [torch.zeros_like(faces) for _ in range(world)]
    dist.all_gather(gathered, faces, group=group)
    n_total = int(offs[-1])
    table = torch.zeros(n_total + 1, dtype=torch.int64, device=dev)
    if rank == 0:
        pairs = []
        for r in range(world - 1):
            a, b = gathered[r][1].cpu().numpy(), gathered[r + 1][0].cpu().numpy()
            both = (a > 0) & (b > 0)
            if both.any():
                pairs.append(np.unique(np.stack([a[both], b[both]], 1), axis=0))
        pr = np.concatenate(pairs) if pairs else np.zeros((0, 2), np.int64)
        rootmap = _union_find_pairs(pr, n_total + 1)
        # renumber roots 1..N in order of first appearance (global raster order)
        uniq, dense = np.unique(rootmap[1:], return_inverse=True)
        table[1:] = torch.from_numpy(dense + 1).to(dev)
    dist.broadcast(table, src=0, group=group)
    out = table[glob.long()].to(torch.int32)
    return out, int(table.max())


def instance_stats(labels: torch.Tensor, n: int, z_offset: int = 0, group=None) -> dict:
    """Per-instance voxel count and centroid (z, y, x), all-reduced across ranks."""
    dev = labels.device
    l = labels.reshape(-1).long()
    fg = l > 0
    Z, Y, X = labels.shape
    idx = torch.nonzero(fg).squeeze(1)
    zz = (idx // (Y * X)).double() + z_offset
    yy = ((idx // X) % Y).double()
    xx = (idx % X).double()
    acc = torch.zeros(4, n + 1, dtype=torch.float64, device=dev)
    lab = l[idx]
    acc[0].index_add_(0, lab, torch.ones_like(zz))
    acc[1].index_add_(0, lab, zz)
    acc[2].index_add_(0, lab, yy)
    acc[3].index_add_(0, lab, xx)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(acc, group=group)
    acc = acc.cpu().numpy()
    c = np.maximum(acc[0, 1:], 1)
    return {"label": list(range(1, n + 1)), "voxels": acc[0, 1:].astype(np.int64).tolist(),
            "centroid_z": (acc[1, 1:] / c).tolist(), "centroid_y": (acc[2, 1:] / c).tolist(),
            "centroid_x": (acc[3, 1:] / c).tolist()}


def analyze_volume(vol: torch.Tensor, predict, tile: int = 512, overlap: int = 64, batch: int = 8,
                   threshold: float = 0.5, min_voxels: int = 300, group=None, gather_labels: bool = False,
                   z_offset: int = 0) -> dict:
    """Single-process (or per-rank) 3-D analysis.  With a process group, ``vol`` is this rank's
    z-slab and results are globally consistent."""
    from ..search.preprocess import percentiles

    v = vol.float()
    sample = v.reshape(1, -1)[:, :: max(1, v.numel() // 4_000_000)]
    p1, p99 = percentiles(sample, (1.0, 99.0))
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        pr = torch.stack([p1, p99]).to(v.device)
        dist.all_reduce(pr, group=group)
        pr /= dist.get_world_size(group)
        p1, p99 = pr[0], pr[1]
    vn = ((v - p1) / (p99 - p1 + 1e-6)).clamp(0, 1)
    prob = slice_probabilities(vn, predict, tile, overlap, batch)
    mask = prob > threshold
    labels, n = label_sharded(mask, group)
    stats = instance_stats(labels, n, z_offset, group)
    keep = np.array(stats["voxels"]) >= min_voxels
    out = {"n_instances": int(keep.sum()), "n_components": n, "volume_shape": list(vol.shape),
           "instances": {k: [x for x, kk in zip(vv, keep) if kk] for k, vv in stats.items()}}
    if gather_labels:
        out["labels"] = labels.cpu().numpy()
    return out
