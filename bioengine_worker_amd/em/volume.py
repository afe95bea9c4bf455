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
    """[Z, Y, X] normalised volume -> foreground probability [Z, Y, X] (slice-wise 2-D model).

    Small slices are predicted ``batch`` slices per call; large slices go through the tiled path
    with the tiles of several slices in one call (the model sees ``batch`` tiles at a time whatever
    the slice size, so a 2048² slice's 25 tiles do not run as 4 under-filled batches)."""
    out = torch.empty(vol.shape, dtype=torch.float32, device=vol.device)
    Z, Y, X = vol.shape
    if Y <= tile and X <= tile:
        for z0 in range(0, Z, batch):
            out[z0:z0 + batch] = predict(vol[z0:z0 + batch][:, None])[:, 0]
        return out
    stride = tile - overlap
    per_slice = len(range(0, Y, stride)) * len(range(0, X, stride))
    k = max(1, batch // per_slice)  # slices whose tiles fill one model batch
    pending: list = []  # tile predictions computed for the current group of slices

    def pooled(t):
        if not pending:
            outs = []
            for i in range(0, cur.shape[0], batch):
                outs.append(predict(cur[i:i + batch]).float())
            pending.extend(torch.cat(outs).split(per_slice))
        return pending.pop(0)

    for z0 in range(0, Z, k):
        zs = list(range(z0, min(Z, z0 + k)))
        tiles = [mito.tile_stack(vol[z], tile, overlap) for z in zs]
        cur = torch.cat(tiles)
        pending.clear()
        for z in zs:
            out[z] = mito.infer_tiled(vol[z], pooled, tile, overlap, per_slice)[0]
    return out


def infer_tiled_3d(vol: torch.Tensor, predict, tile: int = 128, tile_z: int = 32, overlap: int = 16,
                   overlap_z: int = 8, batch: int = 4) -> torch.Tensor:
    """3-D tiled inference with z-overlap blending (SURVEY.md §2.5 K14, 3-D generalisation of the
    reference's 2-D Gaussian tile blend, ``analysis_deployment.py:124-156``).

    ``vol`` [D, H, W] (normalised) is cut into ``tile_z x tile x tile`` blocks with ``overlap_z`` /
    ``overlap`` voxels of overlap (reflect/replicate padded at the far edges); ``predict`` maps
    [B, 1, tz, t, t] -> [B, C, tz, t, t]; predictions are blended with the separable window
    ``exp(-2 z^2) exp(-2 y^2) exp(-2 x^2)`` by the HIP gather-blend kernel (fp32 accumulation, no
    atomics: every output voxel gathers its <= 8 covering tiles).  Returns [C, D, H, W]."""
    D, H, W = vol.shape
    tz, t = min(tile_z, D), min(tile, H, W)
    sz, sxy = max(1, tz - overlap_z), max(1, t - overlap)
    zs, ys, xs = (list(range(0, D, sz)) if D > tz else [0]), list(range(0, H, sxy)), list(range(0, W, sxy))
    pad = (0, max(0, xs[-1] + t - W), 0, max(0, ys[-1] + t - H), 0, max(0, zs[-1] + tz - D))
    big = any(p >= dim for p, dim in zip(pad[::2], (W, H, D)))
    padded = torch.nn.functional.pad(vol[None, None].float(), pad, mode="replicate" if big else "reflect")[0, 0]
    coords = [(z, y, x) for z in zs for y in ys for x in xs]
    outs = []
    for i in range(0, len(coords), batch):
        blk = torch.stack([padded[z:z + tz, y:y + t, x:x + t] for z, y, x in coords[i:i + batch]])[:, None]
        outs.append(predict(blk).float())
    probs = torch.cat(outs).contiguous()
    C = probs.shape[1]
    wz, wxy = mito.gaussian_window(tz).to(vol.device), mito.gaussian_window(t).to(vol.device)
    if vol.is_cuda:
        out = torch.empty(C, D, H, W, dtype=torch.float32, device=vol.device)
        _native.call("be_blend_gather", _native.ptr(probs), C, D, H, W, len(zs), len(ys), len(xs), sxy, sz, tz, t,
                     _native.ptr(wz), _native.ptr(wxy), _native.ptr(wxy), _native.ptr(out), _native.stream(vol.device))
        return out
    return blend3d_reference(probs, D, H, W, zs, ys, xs, tz, t)


def blend3d_reference(probs: torch.Tensor, D: int, H: int, W: int, zs, ys, xs, tz: int, t: int) -> torch.Tensor:
    """float64 scatter-add oracle of :func:`infer_tiled_3d`'s blend."""
    C = probs.shape[1]
    wz, wxy = mito.gaussian_window(tz).double(), mito.gaussian_window(t).double()
    win = wz[:, None, None] * wxy[None, :, None] * wxy[None, None, :]
    acc = torch.zeros(C, D, H, W, dtype=torch.float64)
    wacc = torch.zeros(D, H, W, dtype=torch.float64)
    k = 0
    for z in zs:
        for y in ys:
            for x in xs:
                dz, dy, dx = min(tz, D - z), min(t, H - y), min(t, W - x)
                acc[:, z:z + dz, y:y + dy, x:x + dx] += probs[k, :, :dz, :dy, :dx].double().cpu() * win[:dz, :dy, :dx]
                wacc[z:z + dz, y:y + dy, x:x + dx] += win[:dz, :dy, :dx]
                k += 1
    return (acc / wacc.clamp(min=1e-300)).float()


def _union_find_pairs(pairs: np.ndarray, n: int) -> np.ndarray:
    """Connected components of the label-adjacency graph: root (smallest member) per label 0..n-1."""
    if len(pairs) == 0:
        return np.arange(n)
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    g = coo_matrix((np.ones(len(pairs), np.int8), (pairs[:, 0], pairs[:, 1])), shape=(n, n))
    _, comp = connected_components(g, directed=False)
    first = np.full(comp.max() + 1, n, np.int64)
    np.minimum.at(first, comp, np.arange(n))
    return first[comp]


def _face_pairs(a: torch.Tensor, b: torch.Tensor) -> np.ndarray:
    both = (a > 0) & (b > 0)
    if not bool(both.any()):
        return np.zeros((0, 2), np.int64)
    pr = torch.stack([a[both], b[both]], 1).long()
    return torch.unique(pr, dim=0).cpu().numpy()


#: largest z-chunk the int32 union-find CCL kernel labels in one launch (voxel index < 2^31)
MAX_CCL_VOXELS = 2 ** 31 - 1


def label_local(mask: torch.Tensor, max_voxels: int = MAX_CCL_VOXELS) -> tuple[torch.Tensor, int]:
    """Instance labels 1..n of a [Z, Y, X] mask of any size: z-chunks of < 2^31 voxels are labelled by
    the HIP CCL and chunks touching across a z-face are merged (labels in raster order of first voxel)."""
    Z, Y, X = mask.shape
    cz = max(1, min(Z, max_voxels // max(1, Y * X)))
    if cz >= Z:
        return mito.compact_labels(ccl3d(mask).to(mask.device))
    out = torch.empty(mask.shape, dtype=torch.int32, device=mask.device)
    n = 0
    pairs = []
    for z0 in range(0, Z, cz):
        z1 = min(Z, z0 + cz)
        lab, k = mito.compact_labels(ccl3d(mask[z0:z1]).to(mask.device))
        out[z0:z1] = torch.where(lab > 0, lab + n, lab)
        if z0 > 0:
            pairs.append(_face_pairs(out[z0 - 1], out[z0]))
        n += k
    pr = np.concatenate(pairs) if pairs else np.zeros((0, 2), np.int64)
    if len(pr) == 0:
        return out, n
    root = _union_find_pairs(pr, n + 1)
    uniq, dense = np.unique(root[1:], return_inverse=True)
    table = torch.zeros(n + 1, dtype=torch.int32, device=mask.device)
    table[1:] = torch.from_numpy((dense + 1).astype(np.int32)).to(mask.device)
    for z0 in range(0, Z, cz):  # relabel chunk-wise (no full-volume int64 temporaries)
        z1 = min(Z, z0 + cz)
        out[z0:z1] = table[out[z0:z1].long()]
    return out, int(len(uniq))


def label_sharded(mask_slab: torch.Tensor, group=None) -> tuple[torch.Tensor, int]:
    """Globally consistent instance labels (1..N) for z-slab ``mask_slab`` of this rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    local, n_local = label_local(mask_slab)  # 1..n_local in slab raster order
    if world == 1:
        return local, n_local
    dev = mask_slab.device
    counts = torch.tensor([n_local], dtype=torch.int64, device=dev)
    all_counts = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(all_counts, counts, group=group)
    offs = np.concatenate([[0], np.cumsum([int(c) for c in all_counts])])
    glob = torch.where(local > 0, local + int(offs[rank]), local)
    faces = torch.stack([glob[0], glob[-1]]).to(torch.int64)
    gathered = [torch.zeros_like(faces) for _ in range(world)]
    dist.all_gather(gathered, faces, group=group)
    n_total = int(offs[-1])
    table = torch.zeros(n_total + 1, dtype=torch.int64, device=dev)
    if rank == 0:
        pairs = [_face_pairs(gathered[r][1], gathered[r + 1][0]) for r in range(world - 1)]
        pr = np.concatenate(pairs) if pairs else np.zeros((0, 2), np.int64)
        rootmap = _union_find_pairs(pr, n_total + 1)
        # renumber roots 1..N in order of first appearance (global raster order)
        uniq, dense = np.unique(rootmap[1:], return_inverse=True)
        table[1:] = torch.from_numpy(dense + 1).to(dev)
    dist.broadcast(table, src=0, group=group)
    table32 = table.to(torch.int32)
    out = torch.empty_like(glob)
    cz = max(1, (1 << 28) // max(1, glob[0].numel()))
    for z0 in range(0, glob.shape[0], cz):
        out[z0:z0 + cz] = table32[glob[z0:z0 + cz].long()]
    return out, int(table.max())


def gather_slabs(x: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather z-slabs of possibly different depths into the full [Z, ...] volume on every rank
    (one ``all_gather_into_tensor`` of max-depth-padded slabs — RCCL over xGMI on the GPU node)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return x
    world = dist.get_world_size(group)
    depth = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    depths = [torch.zeros_like(depth) for _ in range(world)]
    dist.all_gather(depths, depth, group=group)
    depths = [int(d) for d in depths]
    zmax = max(depths)
    buf = torch.zeros((zmax,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    buf[: x.shape[0]] = x
    if x.dtype == torch.bool:  # collectives move bytes: ship the mask as uint8
        buf = buf.to(torch.uint8)
    full = torch.empty((world * zmax,) + tuple(x.shape[1:]), dtype=buf.dtype, device=x.device)
    dist.all_gather_into_tensor(full, buf, group=group)
    parts = [full[r * zmax: r * zmax + depths[r]] for r in range(world)]
    out = torch.cat(parts)
    return out.bool() if x.dtype == torch.bool else out


def instance_stats(labels: torch.Tensor, n: int, z_offset: int = 0, group=None) -> dict:
    """Per-instance voxel count and centroid (z, y, x), all-reduced across ranks (z-chunked, so a
    multi-GB label slab never materialises full-size index temporaries)."""
    dev = labels.device
    Z, Y, X = labels.shape
    acc = torch.zeros(4, n + 1, dtype=torch.float64, device=dev)
    cz = max(1, (1 << 27) // max(1, Y * X))
    for z0 in range(0, Z, cz):
        l = labels[z0:z0 + cz].reshape(-1)
        idx = torch.nonzero(l > 0).squeeze(1)
        if idx.numel() == 0:
            continue
        # Segmented sums after a radix sort of the labels instead of index_add_: a large instance
        # sends millions of fp64 atomics to ONE address (a CAS storm that stalls for minutes on a
        # percolating mask); sorted runs reduce with one int64 cumsum per coordinate, exactly.
        lab, perm = torch.sort(l[idx].to(torch.int32))
        idx = idx[perm]
        uniq, counts = torch.unique_consecutive(lab, return_counts=True)
        ends = torch.cumsum(counts, 0) - 1
        u = uniq.long()
        acc[0].index_add_(0, u, counts.double())
        for k, coord in ((1, idx // (Y * X) + z0 + z_offset), (2, (idx // X) % Y), (3, idx % X)):
            cs = torch.cumsum(coord, 0)
            seg = cs[ends] - torch.cat([cs.new_zeros(1), cs[ends[:-1]]])
            acc[k].index_add_(0, u, seg.double())
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(acc, group=group)
    acc = acc.cpu().numpy()
    c = np.maximum(acc[0, 1:], 1)
    return {"label": np.arange(1, n + 1), "voxels": acc[0, 1:].astype(np.int64),
            "centroid_z": acc[1, 1:] / c, "centroid_y": acc[2, 1:] / c, "centroid_x": acc[3, 1:] / c}


def split_instances_sharded(mask: torch.Tensor, group=None, min_size: int = 300, closing_radius: int = 4,
                            min_distance: int = 8) -> tuple[torch.Tensor, int]:
    """Touching objects split by the 3-D marker watershed (:func:`mito.prob_to_instances_3d`) for a
    z-sharded foreground mask: the uint8 mask slabs are gathered onto rank 0 (``dist.gather``; the
    full label volume never exists on the other ranks), rank 0 runs the GPU pipeline on the whole
    volume (a watershed basin can cross any slab face), and each rank gets its label slab back with
    one ``dist.scatter``.  Single process: runs in place.  Returns (this rank's labels, count)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return mito.prob_to_instances_3d(mask, min_size, closing_radius, min_distance)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    depth = torch.tensor([mask.shape[0]], dtype=torch.int64, device=mask.device)
    depths = [torch.zeros_like(depth) for _ in range(world)]
    dist.all_gather(depths, depth, group=group)
    depths = [int(d) for d in depths]
    zmax = max(depths)
    full = gather_to_rank0(mask, group)
    n = torch.zeros(1, dtype=torch.int64, device=mask.device)
    parts = None
    if rank == 0:
        labels, k = mito.prob_to_instances_3d(full, min_size, closing_radius, min_distance)
        n[0] = k
        parts, z = [], 0
        for r in range(world):
            buf = torch.zeros((zmax,) + tuple(mask.shape[1:]), dtype=torch.int32, device=mask.device)
            buf[: depths[r]] = labels[z: z + depths[r]]
            parts.append(buf)
            z += depths[r]
        del labels, full
    mine = torch.empty((zmax,) + tuple(mask.shape[1:]), dtype=torch.int32, device=mask.device)
    dist.scatter(mine, parts, src=0, group=group)
    dist.broadcast(n, src=0, group=group)
    return mine[: mask.shape[0]].contiguous(), int(n.item())


def exchange_halos(x: torch.Tensor, halo: int, group=None) -> tuple[torch.Tensor, int, int]:
    """Point-to-point z-halo exchange between neighbouring slab ranks (RCCL send/recv over xGMI on
    the GPU node, gloo on CPU): returns (``[below-halo | x | above-halo]``, slices received from the
    rank below, slices received from the rank above).  Each neighbour sends min(halo, its depth)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1) or halo <= 0:
        return x, 0, 0
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    depth = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    depths = [torch.zeros_like(depth) for _ in range(world)]
    dist.all_gather(depths, depth, group=group)
    depths = [int(d) for d in depths]
    wire = torch.uint8 if x.dtype == torch.bool else x.dtype
    xs = x.to(wire) if x.dtype == torch.bool else x
    lo = min(halo, depths[rank - 1]) if rank > 0 else 0
    hi = min(halo, depths[rank + 1]) if rank + 1 < world else 0
    below = torch.empty((lo,) + tuple(x.shape[1:]), dtype=wire, device=x.device)
    above = torch.empty((hi,) + tuple(x.shape[1:]), dtype=wire, device=x.device)
    ops = []
    g = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
    if rank > 0:
        ops.append(dist.P2POp(dist.isend, xs[: min(halo, x.shape[0])].contiguous(), g(rank - 1), group))
        ops.append(dist.P2POp(dist.irecv, below, g(rank - 1), group))
    if rank + 1 < world:
        ops.append(dist.P2POp(dist.isend, xs[max(0, x.shape[0] - halo):].contiguous(), g(rank + 1), group))
        ops.append(dist.P2POp(dist.irecv, above, g(rank + 1), group))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    out = torch.cat([below, xs, above])
    return (out.bool() if x.dtype == torch.bool else out), lo, hi


def label_counts(labels: torch.Tensor, n: int) -> torch.Tensor:
    """int64 [n + 1] voxel counts of labels 1..n (index 0 = 0).  On the GPU the LDS-hash chunk
    counter (``be_em_label_counts``): torch.bincount over a 256 x 2048^2 int32 slab of the 3-D EM line
    died with SIGFPE (profiles/r06/rehearsal/), and its per-voxel atomics serialise on large
    components anyway."""
    if labels.is_cuda and labels.dtype == torch.int32 and labels.is_contiguous():
        counts = torch.empty(n + 1, dtype=torch.int32, device=labels.device)
        _native.call("be_em_label_counts", _native.ptr(labels), labels.numel(), _native.ptr(counts), n + 1,
                     _native.stream(labels.device))
        return counts.to(torch.int64)
    cnt = torch.bincount(labels.reshape(-1).long(), minlength=n + 1)[: n + 1].to(torch.int64)
    cnt[0] = 0
    return cnt


def split_instances_halo(mask: torch.Tensor, group=None, min_size: int = 300, closing_radius: int = 4,
                         min_distance: int = 8, halo: int | None = None,
                         timings: dict | None = None) -> tuple[torch.Tensor, int]:
    """Sharded form of :func:`mito.prob_to_instances_3d`: every rank post-processes ITS OWN z-slab
    with a z-halo from its neighbours -- no rank ever holds the whole volume.

    * remove-small: global 6-connected labels (:func:`label_sharded`) + all-reduced voxel counts --
      exact;
    * closing: per z-slice disk, slab-local -- exact;
    * EDT / peak candidates / watershed on ``[halo | slab | halo]`` (P2P halo exchange): the EDT
      inside the slab is exact wherever the nearest background lies within the halo, the
      ``min_distance`` max-filter window needs ``min_distance`` more slices, so the default halo is
      ``closing_radius + 2 * min_distance``;
    * the greedy min-distance thinning (``ensure_spacing``) and the marker numbering are GLOBAL: the
      ranks all-gather their (few) peak candidates, every rank thins the same global list and
      numbers markers in global raster order, exactly like the single-process pipeline -- so labels
      need no seam merge, a basin crossing a slab face carries the same marker id on both sides.
    Returns (this rank's labels, number of instances)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return mito.prob_to_instances_3d(mask, min_size, closing_radius, min_distance, timings=timings)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = mask.device
    halo = closing_radius + 2 * min_distance if halo is None else int(halo)
    depth = torch.tensor([mask.shape[0]], dtype=torch.int64, device=dev)
    depths = [torch.zeros_like(depth) for _ in range(world)]
    dist.all_gather(depths, depth, group=group)
    depths = [int(d) for d in depths]
    z0 = sum(depths[:rank])
    Zg = sum(depths)
    # 1. remove small objects with GLOBAL component sizes
    labels, n = label_sharded(mask, group)
    cnt = label_counts(labels, n)
    dist.all_reduce(cnt, group=group)
    big = cnt >= min_size
    big[0] = False
    binary = big[labels.long()]
    del labels
    # 2. slice-wise closing (slab-local)
    closed = mito.closing_per_slice(binary, closing_radius)
    del binary
    # 3. halo exchange, EDT and peak candidates of the core slices
    ext, lo, hi = exchange_halos(closed, halo, group)
    dmap = mito.edt3d(ext).to(dev)
    core = dmap[lo: lo + mask.shape[0]]
    floor = torch.tensor([float(core.min()) if core.numel() else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(floor, op=dist.ReduceOp.MIN, group=group)
    zyx, vals = mito.peak_candidates3d(dmap, ext, min_distance, lo, lo + mask.shape[0], z0 - lo, Zg,
                                       float(floor.item()))
    # 4. global candidate list -> global greedy thinning -> global raster-order marker ids
    payload = torch.from_numpy(np.concatenate([zyx.astype(np.float64), vals[:, None].astype(np.float64)], 1)
                               if len(zyx) else np.zeros((0, 4))).to(dev)
    m = torch.tensor([payload.shape[0]], dtype=torch.int64, device=dev)
    ms = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(ms, m, group=group)
    mmax = max(1, max(int(v) for v in ms))
    buf = torch.zeros(mmax, 4, dtype=torch.float64, device=dev)
    buf[: payload.shape[0]] = payload
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    allc = torch.cat([bufs[r][: int(ms[r])] for r in range(world)]).cpu().numpy()  # raster order (slabs in z order)
    if len(allc):
        order = np.argsort(-allc[:, 3], kind="stable")  # = single process: stable sort of -value over raster order
        peaks = mito.ensure_spacing(allc[order, :3].astype(np.int64), min_distance).astype(np.int64)
    else:
        peaks = np.zeros((0, 3), np.int64)
    # 5. markers inside the extended slab, numbered by global raster order
    markers = torch.zeros(ext.shape, dtype=torch.int32, device=dev)
    if len(peaks):
        pk = peaks[np.lexsort(peaks.T[::-1])]
        ids = np.arange(1, len(pk) + 1, dtype=np.int32)
        zl = pk[:, 0] - (z0 - lo)
        sel = (zl >= 0) & (zl < ext.shape[0])
        if sel.any():
            loc = torch.from_numpy(np.stack([zl[sel], pk[sel, 1], pk[sel, 2]])).to(dev)
            markers[tuple(loc)] = torch.from_numpy(ids[sel]).to(dev)
    # 6. watershed on the extended slab, keep the core
    if ext.is_cuda:
        lab = mito.watershed_gpu(-dmap, markers, ext)
    else:
        lab = torch.from_numpy(mito.watershed((-dmap).cpu().numpy(), markers.cpu().numpy(), ext.cpu().numpy(), conn=1))
    return lab[lo: lo + mask.shape[0]].to(dev).contiguous(), int(len(peaks))


def analyze_volume(vol: torch.Tensor, predict, tile: int = 512, overlap: int = 64, batch: int = 8,
                   threshold: float = 0.5, min_voxels: int = 300, group=None, gather_labels: bool = False,
                   z_offset: int = 0, gather: str | None = None, timings: bool = False,
                   norm_range: tuple[float, float] | None = None, split_touching: bool = False,
                   closing_radius: int = 4, min_distance: int = 8, predict3d=None, tile_z: int = 32,
                   overlap_z: int = 8, core: tuple[int, int] | None = None, split_halo: int | None = None) -> dict:
    """Single-process (or per-rank) 3-D analysis.  With a process group, ``vol`` is this rank's
    z-slab and results are globally consistent.  ``gather="mask"`` / ``"labels"`` all-gathers the
    stitched foreground mask (uint8) / global instance labels of the whole volume onto every rank
    (``out["mask"]`` / ``out["labels_full"]``, device tensors); ``gather_labels`` returns this
    rank's slab labels as numpy.  ``split_touching`` replaces connected components by the 3-D
    reference post-processing (closing, EDT, peaks, marker watershed) so touching mitochondria
    become separate instances (sharded: :func:`split_instances_halo`, each rank on its own slab).
    ``predict3d`` ([B, 1, tz, t, t] -> [B, C, tz, t, t], a 3-D U-Net) switches inference from
    slice-wise 2-D tiles to 3-D tiles with z-overlap blending (:func:`infer_tiled_3d`); ``core``
    = (lo, hi) crops this rank's slab out of a ``vol`` read with extra z-margin for that context
    (overlap recompute instead of an input halo exchange)."""
    import time

    from ..search.preprocess import percentiles

    marks = [("start", time.perf_counter())]

    def mark(name):
        if timings:
            if vol.is_cuda:
                torch.cuda.synchronize(vol.device)
            marks.append((name, time.perf_counter()))

    v = vol.float()
    if norm_range is not None:  # the whole volume's percentiles, computed by the caller
        p1, p99 = (torch.tensor(float(x), device=v.device) for x in norm_range)
    else:
        p1, p99 = volume_percentiles(v)
    if norm_range is None and dist.is_initialized() and dist.get_world_size(group) > 1:
        pr = torch.stack([p1, p99]).to(v.device)
        dist.all_reduce(pr, group=group)
        pr /= dist.get_world_size(group)
        p1, p99 = pr[0], pr[1]
    vn = ((v - p1) / (p99 - p1 + 1e-6)).clamp(0, 1)
    mark("normalize")
    if predict3d is not None:
        prob = infer_tiled_3d(vn, predict3d, tile=tile, tile_z=tile_z, overlap=overlap, overlap_z=overlap_z,
                              batch=batch)[0]
    else:
        prob = slice_probabilities(vn if core is None else vn[core[0]:core[1]], predict, tile, overlap, batch)
    if predict3d is not None and core is not None:
        prob = prob[core[0]:core[1]]
    mark("inference")
    mask = (prob > threshold).contiguous()
    del prob, vn, v
    split_t: dict | None = {} if timings else None
    if split_touching:
        labels, n = split_instances_halo(mask, group, min_voxels, closing_radius, min_distance, split_halo,
                                         timings=split_t)
    else:
        labels, n = label_sharded(mask, group)
    mark("label")
    stats = instance_stats(labels, n, z_offset, group)
    keep = stats["voxels"] >= min_voxels
    out = {"n_instances": int(keep.sum()), "n_components": n, "volume_shape": list(mask.shape),
           "instances": {k: vv[keep].tolist() for k, vv in stats.items()}}
    mark("stats")
    out["labels_slab_t"] = labels  # this rank's globally consistent slab labels (device tensor)
    if gather_labels:
        out["labels"] = labels.cpu().numpy()
    if gather == "mask":
        out["mask"] = gather_slabs(mask, group)
    elif gather == "labels":
        out["labels_full"] = gather_slabs(labels, group)
    mark("gather")
    if timings:
        out["timings_s"] = {b[0]: round(b[1] - a[1], 4) for a, b in zip(marks, marks[1:])}
        if split_t:
            out["timings_s"]["split_stages"] = split_t
    return out


def volume_percentiles(v, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """p1 / p99 of a strided ~4 M-voxel sample of the volume (torch tensor or numpy / memmap; the
    same sample whether the volume is whole or memory-mapped by every rank of a gang)."""
    from ..search.preprocess import percentiles

    n = int(np.prod(v.shape))
    step = max(1, n // 4_000_000)
    if torch.is_tensor(v):
        sample = v.reshape(1, -1)[:, ::step].float()
    else:
        sample = torch.from_numpy(np.ascontiguousarray(np.asarray(v).reshape(-1)[::step]).astype(np.float32))[None]
    if device is not None:
        sample = sample.to(device)
    return percentiles(sample, (1.0, 99.0))


def gather_to_rank0(x: torch.Tensor, group=None) -> torch.Tensor | None:
    """Stitched full volume on rank 0 only (``dist.gather`` of max-depth-padded slabs): every other
    rank sends its slab once and keeps nothing -- the 2048^3 int32 label volume (34 GB) lands on one
    GPU instead of on all eight.  Returns the volume on rank 0, None elsewhere."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return x
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    depth = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    depths = [torch.zeros_like(depth) for _ in range(world)]
    dist.all_gather(depths, depth, group=group)
    depths = [int(d) for d in depths]
    zmax = max(depths)
    buf = torch.zeros((zmax,) + tuple(x.shape[1:]), dtype=torch.uint8 if x.dtype == torch.bool else x.dtype,
                      device=x.device)
    buf[: x.shape[0]] = x
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0, group=group)
    if rank != 0:
        return None
    out = torch.cat([parts[r][: depths[r]] for r in range(world)])
    return out.bool() if x.dtype == torch.bool else out


class VolumeSource:
    """A [Z, Y, X] volume that every rank reads ONLY its z-range of:

    * ``{"kind": "npy", "path": p}``      -- memory-mapped ``.npy`` (no full read anywhere);
    * ``{"kind": "zarr", "path": p, "array": a}`` -- local zarr v3 directory, chunk reads;
    * ``{"kind": "dataset", "url": u, "array": a, "token": t}`` -- zarr v3 served by the BioEngine
      datasets server, HTTP range reads through :class:`~bioengine_worker_amd.datasets.store.HttpZarrStore`
      (the reference's data plane, ``/root/reference/bioengine/datasets/http_zarr_store.py:31-245``).

    A bare string is a ``.npy`` path (or a ``.zarr`` directory)."""

    def __init__(self, spec):
        if isinstance(spec, (str, bytes)) or hasattr(spec, "__fspath__"):
            p = str(spec)
            spec = {"kind": "zarr" if p.rstrip("/").endswith(".zarr") else "npy", "path": p}
        self.spec = dict(spec)
        self.kind = self.spec["kind"]
        if self.kind == "npy":
            self._mm = np.load(self.spec["path"], mmap_mode="r")
            self.shape = tuple(self._mm.shape)
        elif self.kind in ("zarr", "dataset"):
            self._mm = None
            meta = self._run(self._store().get(self._prefix() + "zarr.json"))
            if meta is None:
                raise FileNotFoundError(f"zarr array not found: {self.spec}")
            from ..datasets.store import zarr_shape

            self.shape = zarr_shape(meta)
        else:
            raise ValueError(f"unknown volume source kind {self.kind!r}")
        if len(self.shape) != 3:
            raise ValueError(f"expected a [Z, Y, X] volume, got shape {self.shape}")

    def _prefix(self) -> str:
        a = (self.spec.get("array") or "").strip("/")
        return f"{a}/" if a else ""

    def _store(self):
        from ..datasets.store import HttpZarrStore, LocalZarrStore

        if self.kind == "zarr":
            return LocalZarrStore(self.spec["path"])
        return HttpZarrStore(self.spec["url"], token=self.spec.get("token"))

    @staticmethod
    def _run(coro):
        import asyncio

        return asyncio.run(coro)

    def read(self, z0: int, z1: int) -> np.ndarray:
        z0, z1 = max(0, z0), min(self.shape[0], z1)
        if self.kind == "npy":
            return np.ascontiguousarray(self._mm[z0:z1])
        from ..datasets.store import read_zarr_array

        async def go():
            st = self._store()
            try:
                return await read_zarr_array(st, self.spec.get("array") or "",
                                             (slice(z0, z1), slice(0, self.shape[1]), slice(0, self.shape[2])))
            finally:
                await st.close()

        return self._run(go())

    def percentiles(self, device=None) -> tuple[torch.Tensor, torch.Tensor]:
        """p1 / p99 of a deterministic sample, identical on every rank: the strided flat sample of
        a memory-mapped ``.npy``; for zarr sources up to 16 evenly spaced z-slices, strided."""
        if self.kind == "npy":
            return volume_percentiles(self._mm, device)
        Z = self.shape[0]
        zs = sorted(set(int(round(z)) for z in np.linspace(0, Z - 1, min(16, Z))))
        sl = np.stack([self.read(z, z + 1)[0] for z in zs])
        return volume_percentiles(sl, device)


def probability_identity(tiles: torch.Tensor) -> torch.Tensor:
    """``predict`` for inputs that are already foreground probabilities (normalised 0..1)."""
    return tiles


def gang_analyze_volume(rank: int, world: int, volume_path=None, out_path: str = "", model_root: str | None = None,
                        tile: int = 512,
                        overlap: int = 64, batch: int = 8, threshold: float = 0.5, min_voxels: int = 300,
                        gather: str = "rank0", volume=None, split_touching: bool = False, closing_radius: int = 4,
                        min_distance: int = 8, model3d_root: str | None = None, tile_z: int = 32,
                        overlap_z: int = 8) -> dict:
    """Gang target (``serve/gang.py``): rank r reads ONLY its z-slab of the volume (``volume``: a
    :class:`VolumeSource` spec -- memory-mapped ``.npy``, local zarr, or a datasets-server zarr over
    HTTP; ``volume_path``: a ``.npy`` path), runs tiled inference (slice-wise 2-D, or 3-D tiles with
    a z-margin recomputed instead of exchanged when ``model3d_root`` is given) and labelling; the
    ranks agree on global labels over the process group (RCCL on the GPU node).  ``split_touching``
    runs the reference post-processing sharded (:func:`split_instances_halo`).  ``gather``:
    ``"rank0"`` stitches the label volume on rank 0 and writes ``out_path`` (``.npy``);
    ``"sharded"`` leaves each slab where it was computed and writes ``<out_path>.rank<r>.npy`` + the
    z offsets; ``"none"`` keeps only the statistics."""
    import json
    import time

    from ..bioimageio.runner import PredictionPipeline

    group = None
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t0 = time.perf_counter()
    src = VolumeSource(volume if volume is not None else volume_path)
    Z = src.shape[0]
    z0, z1 = slab_bounds(Z, rank, world)
    predict, predict3d, core, margin = probability_identity, None, None, 0
    if model3d_root:
        pipe3 = PredictionPipeline(model3d_root, device=dev)
        predict3d = lambda t: next(iter(pipe3.predict_tensors(t).values()))
        margin = max(overlap_z, tile_z // 2)
    elif model_root:
        pipe = PredictionPipeline(model_root, device=dev)
        predict = lambda t: next(iter(pipe.predict_tensors(t).values()))
    # else: the volume already is a probability map (e.g. from an earlier pass): identity "model"
    za, zb = max(0, z0 - margin), min(Z, z1 + margin)
    slab = torch.from_numpy(src.read(za, zb)).to(dev)
    if margin:
        core = (z0 - za, z0 - za + (z1 - z0))
    p1, p99 = src.percentiles(dev)  # identical on every rank and to the single-GPU path
    res = analyze_volume(slab, predict, tile, overlap, batch, threshold, min_voxels, group=group, z_offset=z0,
                         timings=True, norm_range=(float(p1), float(p99)), split_touching=split_touching,
                         closing_radius=closing_radius, min_distance=min_distance, predict3d=predict3d,
                         tile_z=tile_z, overlap_z=overlap_z, core=core)
    t_an = time.perf_counter()
    out = {"rank": rank, "z_range": [z0, z1], "n_instances": res["n_instances"], "timings_s": res["timings_s"]}
    if gather == "rank0":
        full = gather_to_rank0(res["labels_slab_t"], group)
        if rank == 0:
            np.save(out_path, full.cpu().numpy())
    elif gather == "sharded":
        np.save(f"{out_path}.rank{rank}.npy", res["labels_slab_t"].cpu().numpy())
        if rank == 0:
            with open(f"{out_path}.manifest.json", "w") as f:
                json.dump({"world": world, "z_ranges": [list(slab_bounds(Z, r, world)) for r in range(world)],
                           "files": [f"{out_path}.rank{r}.npy" for r in range(world)]}, f)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    out["gather_s"] = round(time.perf_counter() - t_an, 4)
    out["total_s"] = round(time.perf_counter() - t0, 4)
    if rank == 0:
        out.update(n_components=res["n_components"], volume_shape=list(src.shape), instances=res["instances"],
                   split_touching=bool(split_touching), inference="tiled3d" if predict3d is not None else "slice2d")
    return out
