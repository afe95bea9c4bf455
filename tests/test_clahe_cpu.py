"""CLAHE oracle (bioengine_worker_amd/ops/clahe.py) — properties of OpenCV's 8-bit algorithm.
cv2 is not installed here, so cv2 parity itself is unpinned; these pin the algorithm's defining
steps (clip limit, residual redistribution, LUT rounding, bilinear blend, reflect-101 padding)."""
import numpy as np

from bioengine_worker_amd.ops.clahe import clahe_u8, clahe_u8_ref, to_gray_u8


def test_uniform_tile_hand_computed():
    # 64x64 / 16x16 grid -> 4x4 tiles (area 16): limit = max(1, int(3*16/256)) = 1; a constant 77
    # clips 15 counts: batch 0, residual 15, step 256 // 15 = 17 -> bins 0, 17, ..., 238 get +1.
    # cumsum at 77 = 5 (bins 0..68) + 1 = 6 -> round(6 * 255 / 16) = 96 everywhere.
    out = clahe_u8_ref(np.full((64, 64), 77, np.uint8))
    assert np.all(out == 96)


def test_monotone_and_clip_bounds():
    rng = np.random.default_rng(0)
    img = (rng.random((128, 128)) ** 3 * 255).astype(np.uint8)
    out = clahe_u8_ref(img)
    # pixels that share bilinear weights (same position, different images) map monotonically
    img2 = np.minimum(img.astype(int) + 10, 255).astype(np.uint8)
    img2[:, :] = img  # same histograms ...
    img2[64, 64] = min(255, int(img[64, 64]) + 1)  # ... except one count moved up by one level
    assert int(clahe_u8_ref(img2)[64, 64]) >= int(out[64, 64])
    # contrast enhancement spreads a dark-skewed histogram
    assert out.std() > 0.9 * img.std() and out.mean() > img.mean()
    # a higher clip limit enhances at least as strongly (further from identity on average)
    lo = clahe_u8_ref(img, clip=1.0)
    hi = clahe_u8_ref(img, clip=8.0)
    assert np.abs(hi.astype(int) - img).mean() >= np.abs(lo.astype(int) - img).mean()


def test_reflect101_padding_matches_explicit_padding():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (50, 70), dtype=np.uint8)
    out = clahe_u8_ref(img)
    # extend by hand (reflect-101 == numpy "reflect") to 64 x 80 and run on the divisible size:
    # the LUTs are identical, so the interior blend agrees wherever tile sizes are the same
    ext = np.pad(img, ((0, 14), (0, 10)), mode="reflect")
    out_ext = clahe_u8_ref(ext)
    assert out.shape == (50, 70)
    np.testing.assert_array_equal(out, out_ext[:50, :70])


def test_to_gray_u8_reference_semantics():
    rgb = np.zeros((3, 10, 12), np.uint8)
    rgb[0] = 100
    rgb[1] = 50
    rgb[2] = 200
    g = to_gray_u8(rgb)  # CHW detected -> luminance
    assert g.shape == (10, 12) and g.dtype == np.uint8
    assert int(g[0, 0]) == int(np.float32(0.299 * 100 + 0.587 * 50 + 0.114 * 200))
    f = np.linspace(0, 1000, 120, dtype=np.float32).reshape(10, 12)
    g2 = to_gray_u8(f)
    assert g2.min() == 0 and g2.max() == 255
    import torch

    t = clahe_u8(torch.from_numpy(g2))
    np.testing.assert_array_equal(t.numpy(), clahe_u8_ref(g2))
