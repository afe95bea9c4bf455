"""Instance-segmentation metrics: IoU-matched average precision.

The reference evaluates a fine-tuned model on the held-out images with cellpose's
``metrics.average_precision(masks_true, masks_pred, threshold=[0.5, 0.75, 0.9])`` and reports the
image mean as ``InstanceMetrics(ap_0_5, ap_0_75, ap_0_9, n_true, n_pred)``
(apps/cellpose-finetuning/main.py:1980-2029).  Same definitions here:

* overlap[i, j] = pixels with true label i and predicted label j (a joint histogram — one bincount,
  on the GPU for device tensors);
* IoU = overlap / (area_true + area_pred - overlap), background row/column dropped;
* true positives at threshold t = an optimal one-to-one matching (Hungarian, scipy) maximising
  "IoU >= t" first and total IoU second (cost = -(iou >= t) - iou / (2 * min(n_true, n_pred)));
* AP = tp / (tp + fp + fn) per image, fp = n_pred - tp, fn = n_true - tp (NaN when both are empty).
Labels are the integers in the masks (0 = background); n_true / n_pred are the label maxima, as in
cellpose.
"""
from __future__ import annotations

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment

DEFAULT_THRESHOLDS = (0.5, 0.75, 0.9)


def label_overlap(mt, mp) -> np.ndarray:
    """[n_true + 1, n_pred + 1] int64 pixel overlap counts."""
    if isinstance(mt, torch.Tensor) or isinstance(mp, torch.Tensor):
        t = torch.as_tensor(mt).long().reshape(-1)
        p = torch.as_tensor(mp).long().reshape(-1).to(t.device)
        nt, np_ = int(t.max().item()) + 1, int(p.max().item()) + 1
        return torch.bincount(t * np_ + p, minlength=nt * np_).reshape(nt, np_).cpu().numpy()
    t = np.asarray(mt).astype(np.int64).ravel()
    p = np.asarray(mp).astype(np.int64).ravel()
    nt, np_ = int(t.max()) + 1, int(p.max()) + 1
    return np.bincount(t * np_ + p, minlength=nt * np_).reshape(nt, np_)


def intersection_over_union(mt, mp) -> np.ndarray:
    ov = label_overlap(mt, mp).astype(np.float64)
    area_t = ov.sum(1, keepdims=True)
    area_p = ov.sum(0, keepdims=True)
    with np.errstate(invalid="ignore", divide="ignore"):
        iou = ov / (area_t + area_p - ov)
    iou[np.isnan(iou)] = 0.0
    return iou


def true_positive(iou: np.ndarray, th: float) -> int:
    n_min = min(iou.shape)
    if n_min == 0:
        return 0
    costs = -(iou >= th).astype(np.float64) - iou / (2 * n_min)
    ti, pi = linear_sum_assignment(costs)
    return int((iou[ti, pi] >= th).sum())


def average_precision(masks_true, masks_pred, threshold=DEFAULT_THRESHOLDS):
    """Returns (ap, tp, fp, fn) each [n_images, n_thresholds] (single arrays -> [n_thresholds])."""
    single = not isinstance(masks_true, (list, tuple))
    if single:
        masks_true, masks_pred = [masks_true], [masks_pred]
    ths = [threshold] if np.isscalar(threshold) else list(threshold)
    n = len(masks_true)
    ap = np.zeros((n, len(ths)), np.float32)
    tp = np.zeros((n, len(ths)), np.int64)
    fp = np.zeros((n, len(ths)), np.int64)
    fn = np.zeros((n, len(ths)), np.int64)
    for i, (mt, mp) in enumerate(zip(masks_true, masks_pred)):
        n_true = int(torch.as_tensor(mt).max().item()) if np.asarray(mt.shape).prod() else 0
        n_pred = int(torch.as_tensor(mp).max().item()) if np.asarray(mp.shape).prod() else 0
        if n_pred > 0 and n_true > 0:
            iou = intersection_over_union(mt, mp)[1:, 1:]
            for k, th in enumerate(ths):
                tp[i, k] = true_positive(iou, th)
        fp[i] = n_pred - tp[i]
        fn[i] = n_true - tp[i]
        with np.errstate(invalid="ignore", divide="ignore"):
            ap[i] = tp[i] / (tp[i] + fp[i] + fn[i]).astype(np.float32)
    if single:
        return ap[0], tp[0], fp[0], fn[0]
    return ap, tp, fp, fn


def instance_metrics(masks_true, masks_pred, threshold=DEFAULT_THRESHOLDS) -> dict:
    """The reference's InstanceMetrics document (image-mean AP at 0.5 / 0.75 / 0.9 + label counts)."""
    ap, _, _, _ = average_precision(list(masks_true), list(masks_pred), threshold)
    with np.errstate(all="ignore"):
        mean_ap = np.nanmean(ap, axis=0) if len(ap) else np.full(len(threshold), np.nan)
    out = {f"ap_{str(t).replace('.', '_')}": (round(float(m), 4) if np.isfinite(m) else None)
           for t, m in zip(threshold, mean_ap)}
    out["n_true"] = int(sum(int(torch.as_tensor(m).max().item()) for m in masks_true))
    out["n_pred"] = int(sum(int(torch.as_tensor(m).max().item()) for m in masks_pred))
    return out
