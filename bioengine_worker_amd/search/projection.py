"""2-D projection of embeddings for the UMAP preview (reference index_manager.py:185-271, K23).

umap-learn is used when importable; otherwise (as in this offline image) the projection is a
GPU PCA (``torch.pca_lowrank``) — the reference falls back to PCA the same way.  Results are
cached in ``umap_cache.npz`` (plain arrays; no pickles)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch


def palette(n: int) -> list[str]:
    import colorsys

    out = []
    for i in range(max(n, 1)):
        r, g, b = colorsys.hsv_to_rgb((i * 0.618033988749895) % 1.0, 0.65, 0.9)
        out.append("#%02x%02x%02x" % (int(r * 255), int(g * 255), int(b * 255)))
    return out


def project_2d(vecs: np.ndarray, seed: int = 42) -> tuple[np.ndarray, str]:
    try:
        from umap import UMAP  # noqa: F401

        return UMAP(n_neighbors=15, min_dist=0.1, metric="cosine", random_state=seed).fit_transform(vecs), "umap"
    except ImportError:
        dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        x = torch.from_numpy(np.asarray(vecs, np.float32)).to(dev)
        x = x - x.mean(0, keepdim=True)
        torch.manual_seed(seed)
        _, _, V = torch.pca_lowrank(x, q=min(6, x.shape[1]), center=False)
        return (x @ V[:, :2]).cpu().numpy(), "pca"


def compute_projection(index, labels: list[str] | None, cache_path: Path, n_samples: int = 10_000, seed: int = 42,
                       force: bool = False, tag: str = "") -> dict:
    cache_path = Path(cache_path)
    if cache_path.exists() and not force:
        d = np.load(cache_path)
        return {"x": d["x"].tolist(), "y": d["y"].tolist(), "labels": [str(s) for s in d["labels"]],
                "colors": [str(s) for s in d["colors"]], "n_total": int(d["n_total"]), "sample_idx": d["idx"].tolist(),
                "method": str(d["method"])}
    n_total = index.ntotal if index is not None else 0
    if n_total == 0:
        return {"x": [], "y": [], "labels": [], "colors": [], "n_total": 0, "sample_idx": [], "method": "none"}
    n = min(n_samples, n_total)
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(n_total, size=n, replace=False))
    coords, method = project_2d(index.reconstruct_batch(idx), seed)
    lab = [str(labels[i]) if labels is not None and i < len(labels) else "unknown" for i in idx]
    uniq = sorted(set(lab))
    cmap = dict(zip(uniq, palette(len(uniq))))
    col = [cmap[s] for s in lab]
    cache_path.parent.mkdir(parents=True, exist_ok=True)
    np.savez(cache_path, x=coords[:, 0], y=coords[:, 1], labels=np.array(lab, dtype=str), colors=np.array(col, dtype=str),
             n_total=np.array(n_total), idx=idx, method=np.array(method))
    return {"x": coords[:, 0].tolist(), "y": coords[:, 1].tolist(), "labels": lab, "colors": col, "n_total": n_total,
            "sample_idx": idx.tolist(), "method": method}
