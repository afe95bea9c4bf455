"""HIP training kernels vs PyTorch fp32 references."""
import math

import pytest
import torch

from bioengine_worker_amd.ops import train_ops


@pytest.mark.gpu
def test_adamw_matches_torch(gpu):
    torch.manual_seed(0)
    n = 10_003
    p0 = torch.randn(n)
    p_ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([p_ref], lr=1e-3, weight_decay=0.1)
    p = p0.clone().to(gpu)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    pbf = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    for step in range(1, 6):
        g = torch.randn(n)
        p_ref.grad = g.clone()
        opt.step()
        train_ops.adamw_flat_(p, (2 * g).to(gpu), m, v, lr=1e-3, step=step, weight_decay=0.1, grad_scale=0.5, p_bf16=pbf)
    assert (p.cpu() - p_ref.detach()).abs().max().item() < 1e-5
    assert (pbf.float().cpu() - p_ref.detach()).abs().max().item() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_seg_loss_fwd_bwd(gpu, dtype):
    torch.manual_seed(0)
    y = torch.randn(3, 3, 40, 56)
    lbl = torch.cat([(torch.rand(3, 1, 40, 56) > 0.5).float() * 3, torch.randn(3, 2, 40, 56) * 0.5], 1)
    yr = y.clone().requires_grad_(True)
    lr = train_ops.seg_loss_ref(yr, lbl)
    lr.backward()
    yg = y.to(gpu, dtype).requires_grad_(True)
    lg = train_ops.seg_loss(yg, lbl.to(gpu))
    lg.backward()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert abs(lg.item() - lr.item()) < tol * max(1, abs(lr.item()))
    assert (yg.grad.float().cpu() - yr.grad).abs().max().item() < tol * yr.grad.abs().max().item() + 1e-7


@pytest.mark.gpu
def test_affine_warp_matches_reference(gpu):
    torch.manual_seed(0)
    img = torch.rand(3, 2, 80, 96)
    lbl = torch.cat([torch.randint(0, 5, (3, 1, 80, 96)).float(), torch.randn(3, 2, 80, 96)], 1)
    aff, flip, _ = train_ops.random_affine_params(3, 80, 96, xy=(64, 64), scale_range=0.5,
                                                  generator=torch.Generator().manual_seed(3))
    oi_r, ol_r = train_ops.affine_warp_ref(img, lbl, aff, flip, 64, 64)
    oi, ol = train_ops.affine_warp(img.to(gpu), lbl.to(gpu), aff, flip, 64, 64)
    assert (oi.cpu() - oi_r).abs().max().item() < 1e-4
    assert (ol[:, 1:].cpu() - ol_r[:, 1:]).abs().max().item() < 1e-4
    # nearest channel: allow rare rounding-boundary disagreements
    assert (ol[:, 0].cpu() != ol_r[:, 0]).float().mean().item() < 0.01


@pytest.mark.gpu
def test_trainer_step_decreases_loss(gpu):
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    tr = build_trainer(TrainConfig(batch_size=4, bsize=128, lr=2e-3, weight_decay=0.0), device=gpu)
    batch = synthetic_train_batch(4, 128, device=gpu)
    tr.gen.manual_seed(0)
    first = [float(tr.step(*batch)) for _ in range(3)]
    for _ in range(20):
        last = float(tr.step(*batch))
    assert math.isfinite(last) and last < first[0]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 256), (100, 130), (37, 530)])
def test_clahe_kernel_bit_exact(gpu, shape):
    """HIP CLAHE == numpy oracle (incl. reflect-101 padding for sizes not divisible by the grid)."""
    import numpy as np

    from bioengine_worker_amd.ops.clahe import clahe_u8, clahe_u8_ref

    rng = np.random.default_rng(sum(shape))
    imgs = np.stack([(rng.random(shape) ** (1 + i) * 255).astype(np.uint8) for i in range(3)])
    out = clahe_u8(torch.from_numpy(imgs).to(gpu)).cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(out[i], clahe_u8_ref(imgs[i]))
