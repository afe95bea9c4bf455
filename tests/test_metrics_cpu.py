"""Instance AP metrics (bioengine_worker_amd/cellpose/metrics.py) on hand-built label images."""
import numpy as np
import torch

from bioengine_worker_amd.cellpose.metrics import (average_precision, instance_metrics, intersection_over_union,
                                                   label_overlap, true_positive)


def _boxes(shape, boxes):
    m = np.zeros(shape, np.int32)
    for k, (y0, y1, x0, x1) in enumerate(boxes, start=1):
        m[y0:y1, x0:x1] = k
    return m


def test_perfect_and_empty():
    mt = _boxes((40, 40), [(0, 10, 0, 10), (20, 30, 20, 30)])
    ap, tp, fp, fn = average_precision(mt, mt.copy())
    assert np.all(ap == 1) and np.all(tp == 2) and np.all(fp == 0) and np.all(fn == 0)
    ap, tp, fp, fn = average_precision(mt, np.zeros_like(mt))
    assert np.all(ap == 0) and np.all(fn == 2)
    ap, *_ = average_precision(np.zeros_like(mt), np.zeros_like(mt))
    assert np.all(np.isnan(ap))


def test_iou_thresholds_hand_computed():
    mt = _boxes((50, 50), [(0, 10, 0, 10), (20, 30, 20, 30)])
    # pred 1: shifted by 2 columns -> IoU = 80 / 120 = 0.667 (passes 0.5 only)
    # pred 2: exact; pred 3: a false positive
    mp = _boxes((50, 50), [(0, 10, 2, 12), (20, 30, 20, 30), (40, 45, 40, 45)])
    iou = intersection_over_union(mt, mp)[1:, 1:]
    assert abs(iou[0, 0] - 80 / 120) < 1e-12 and iou[1, 1] == 1.0
    ap, tp, fp, fn = average_precision(mt, mp, threshold=[0.5, 0.75, 0.9])
    np.testing.assert_array_equal(tp, [2, 1, 1])
    np.testing.assert_array_equal(fp, [1, 2, 2])
    np.testing.assert_array_equal(fn, [0, 1, 1])
    np.testing.assert_allclose(ap, [2 / 3, 1 / 4, 1 / 4], rtol=1e-6)


def test_matching_is_one_to_one():
    mt = _boxes((20, 40), [(0, 20, 0, 20)])
    mp = _boxes((20, 40), [(0, 20, 0, 12), (0, 20, 12, 20)])  # one true split into two predictions
    iou = intersection_over_union(mt, mp)[1:, 1:]
    assert true_positive(iou, 0.5) == 1 and true_positive(iou, 0.7) == 0


def test_overlap_torch_and_numpy_agree_and_instance_doc():
    rng = np.random.default_rng(0)
    mt = rng.integers(0, 6, (30, 30)).astype(np.int32)
    mp = rng.integers(0, 4, (30, 30)).astype(np.int32)
    np.testing.assert_array_equal(label_overlap(mt, mp), label_overlap(torch.from_numpy(mt), torch.from_numpy(mp)))
    doc = instance_metrics([mt, mt], [mt, mp])
    assert set(doc) == {"ap_0_5", "ap_0_75", "ap_0_9", "n_true", "n_pred"}
    assert doc["n_true"] == 2 * int(mt.max()) and doc["n_pred"] == int(mt.max()) + int(mp.max())
    assert 0.5 <= doc["ap_0_5"] <= 1.0
