"""CPU oracle sanity: flows from synthetic label disks recover the same instances."""
import numpy as np
import pytest

from bioengine_worker_amd.cellpose import reference as ref


def disk_labels(H=96, W=96, n=6, seed=0):
    rng = np.random.default_rng(seed)
    M = np.zeros((H, W), np.int32)
    yy, xx = np.mgrid[0:H, 0:W]
    k = 0
    for _ in range(200):
        if k == n:
            break
        cy, cx, r = rng.uniform(12, H - 12), rng.uniform(12, W - 12), rng.uniform(6, 10)
        d = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
        if (M[d] > 0).any():
            continue
        k += 1
        M[d] = k
    return M


def flows_from_labels(M):
    mu = ref.masks_to_flows(M)
    dP = 5.0 * mu
    cellprob = np.where(M > 0, 5.0, -5.0).astype(np.float32)
    return dP.astype(np.float32), cellprob


@pytest.mark.unit
def test_masks_roundtrip_recovers_instances():
    M = disk_labels()
    dP, cp = flows_from_labels(M)
    out = ref.compute_masks(dP, cp, niter=200)
    assert out.max() == M.max()
    # every true instance maps to exactly one predicted instance with high IoU
    for lab in range(1, M.max() + 1):
        pred = out[M == lab]
        vals, counts = np.unique(pred[pred > 0], return_counts=True)
        assert len(vals) >= 1 and counts.max() / (M == lab).sum() > 0.9


@pytest.mark.unit
def test_fill_holes_and_min_size():
    M = np.zeros((40, 40), np.int32)
    M[5:20, 5:20] = 1
    M[10:13, 10:13] = 0  # hole
    M[30:32, 30:32] = 2  # tiny (4 px) -> removed
    out = ref.fill_holes_and_remove_small_masks(M, min_size=15)
    assert out.max() == 1
    assert (out[10:13, 10:13] == 1).all()
    assert (out[30:32, 30:32] == 0).all()


@pytest.mark.unit
def test_tiles_cover_and_blend_identity():
    img = np.random.default_rng(0).standard_normal((3, 300, 260)).astype(np.float32)
    tiles, ys, xs = ref.make_tiles(img, 224, 0.1)
    out = ref.average_tiles(tiles, ys, xs, 300, 260)
    np.testing.assert_allclose(out, img, atol=1e-5)
