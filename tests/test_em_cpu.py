"""EM post-processing host runtime (C++ watershed, peak spacing) vs Python oracles; blending oracle;
regionprops formulas."""
import heapq

import numpy as np

from bioengine_worker_amd.em import mito


def _watershed_py(img, markers, mask):
    H, W = img.shape
    out = np.where(mask, markers, 0).astype(np.int32)
    hp = [(img[y, x], 0, y * W + x) for y, x in zip(*np.nonzero(out))]
    heapq.heapify(hp)
    age = 1
    while hp:
        v, a, i = heapq.heappop(hp)
        y, x = divmod(i, W)
        for dy, dx in ((-1, 0), (0, -1), (0, 1), (1, 0)):
            yy, xx = y + dy, x + dx
            if 0 <= yy < H and 0 <= xx < W and mask[yy, xx] and not out[yy, xx]:
                out[yy, xx] = out[y, x]
                heapq.heappush(hp, (img[yy, xx], age, yy * W + xx))
                age += 1
    return out


def test_watershed_matches_heap_oracle():
    from scipy import ndimage

    rng = np.random.default_rng(0)
    mask = np.zeros((80, 90), bool)
    yy, xx = np.mgrid[0:80, 0:90]
    for cy, cx, r in ((20, 20, 14), (30, 40, 15), (60, 60, 18), (55, 25, 10)):
        mask |= (yy - cy) ** 2 + (xx - cx) ** 2 < r * r
    dist = ndimage.distance_transform_edt(mask).astype(np.float32) + rng.random((80, 90)).astype(np.float32) * 1e-3
    markers = np.zeros_like(mask, np.int32)
    for k, (cy, cx) in enumerate(((20, 20), (30, 40), (60, 60), (55, 25))):
        markers[cy, cx] = k + 1
    got = mito.watershed(-dist, markers, mask)
    ref = _watershed_py(-dist, markers, mask)
    assert (got == ref).all()
    assert set(np.unique(got)) == {0, 1, 2, 3, 4}


def test_ensure_spacing_greedy():
    rng = np.random.default_rng(1)
    pts = rng.integers(0, 100, (300, 2))
    kept = mito.ensure_spacing(pts, 8)
    # oracle: greedy in order, reject later points with Chebyshev distance < 8 from a kept one
    ref = []
    rej = np.zeros(len(pts), bool)
    for i in range(len(pts)):
        if rej[i]:
            continue
        ref.append(pts[i])
        d = np.abs(pts - pts[i]).max(1)
        rej |= d < 8
    assert np.array_equal(kept, np.array(ref))


def test_blend_reference_is_partition_of_unity():
    probs = np.ones((4, 1, 64, 64), np.float32)
    import torch

    out = mito.blend_reference(torch.from_numpy(probs), 100, 100, [0, 48], [0, 48], 64)
    assert np.allclose(out.numpy(), 1.0, atol=1e-6)


def test_region_properties_cpu_ellipse():
    lab = np.zeros((100, 100), np.int32)
    yy, xx = np.mgrid[0:100, 0:100]
    lab[((yy - 50) / 30.0) ** 2 + ((xx - 40) / 10.0) ** 2 < 1] = 1
    p = mito.region_properties(lab, 5.0, device="cpu")
    assert p["label"] == [1] and abs(p["centroid_y"][0] - 50) < 0.5 and abs(p["centroid_x"][0] - 40) < 0.5
    assert 2.7 < p["aspect_ratio"][0] < 3.3 and 0.9 < p["eccentricity"][0] < 0.97
