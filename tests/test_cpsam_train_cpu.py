"""Cellpose-SAM training engine (train/cpsam_engine.py) on CPU: the hand-written forward/backward
(every op on its fp32 PyTorch reference) must match PyTorch autograd through the CPSAM module, with
per-sample stochastic depth active."""
import copy

import pytest
import torch

from bioengine_worker_amd.models.cpsam import CPSAM
from bioengine_worker_amd.ops import train_ops
from bioengine_worker_amd.parallel.ddp import FlatParams
from bioengine_worker_amd.train.cpsam_engine import CPSAMTrainEngine, stochastic_depth_keep


def _small(seed=0):
    torch.manual_seed(seed)
    net = CPSAM(dim=128, depth=3, heads=2, ps=8, bsize=64, rdrop=0.4).randomize_(seed)
    with torch.no_grad():  # non-trivial norms / biases so their gradients are exercised
        for n, p in net.named_parameters():
            if p.requires_grad and ("norm" in n or "neck.1" in n or "neck.3" in n or n.endswith("bias")):
                p.add_(0.1 * torch.randn_like(p))
    return net


@pytest.mark.unit
def test_cpsam_engine_matches_autograd_cpu():
    torch.set_num_threads(4)
    B = 2
    net = _small()
    ref = copy.deepcopy(net).train()
    x = torch.randn(B, 2, 64, 64)
    lbl = torch.zeros(B, 3, 64, 64)
    lbl[:, 0] = (torch.rand(B, 64, 64) > 0.6).float()
    lbl[:, 1:] = torch.randn(B, 2, 64, 64) * 0.3
    keep = stochastic_depth_keep(B, 3, 0.8, "cpu", torch.Generator().manual_seed(3))
    keep[0, 1] = 0.0  # make sure at least one block is dropped for one sample
    keep[1, 1] = 1.0

    # autograd oracle
    x3 = torch.cat([x, torch.zeros(B, 1, 64, 64)], 1)
    y_ref = ref(x3, keep=keep)[0]
    loss_ref = train_ops.seg_loss_ref(y_ref, lbl)
    loss_ref.backward()

    fp = FlatParams(net, "cpu")
    eng = CPSAMTrainEngine(net, fp, B, "cpu")
    loss = eng.loss_and_backward(x, lbl, keep)
    assert abs(float(loss) - float(loss_ref)) < 1e-4 * max(1.0, abs(float(loss_ref)))
    ref_grads = dict(ref.named_parameters())
    worst = 0.0
    for name, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g_ref = ref_grads[name].grad
        assert g_ref is not None, name
        err = (p.grad - g_ref).abs().max().item() / max(g_ref.abs().max().item(), 1e-8)
        worst = max(worst, err)
        assert err < 1e-3, f"{name}: rel err {err:.2e}"
    # dropped block: sample 0 contributes nothing, sample 1 does -> gradients are non-zero
    assert net.encoder.blocks[1].mlp.lin1.weight.grad.abs().sum() > 0


@pytest.mark.unit
def test_stochastic_depth_schedule():
    keep = stochastic_depth_keep(4096, 24, 0.4, "cpu", torch.Generator().manual_seed(0))
    drop = 1 - keep.mean(0)
    assert drop[0] == 0.0
    assert abs(float(drop[-1]) - 0.4) < 0.03
    assert abs(float(drop[12]) - 0.4 * 12 / 23) < 0.03


def test_relpos_oracles_match_engine_batched_gemms():
    """vit_train.relpos_*_ref (the oracle of relpos.hip) == the engine's torch formulation."""
    from bioengine_worker_amd.ops import vit_train as vt

    net = CPSAM(dim=128, depth=1, heads=2, ps=8, bsize=64).randomize_(0)
    eng = CPSAMTrainEngine(net, FlatParams(net, "cpu"), 2, "cpu")
    torch.manual_seed(0)
    B, g, H, c = eng.B, eng.g, eng.H, eng.hd
    q = torch.randn(B, g * g, H, c)
    Rh, Rw = torch.randn(g, g, c), torch.randn(g, g, c)
    rh, rw = eng._rel_terms(q, Rh, Rw)
    rh2, rw2 = vt.relpos_fwd_ref(q, Rh, Rw)
    assert torch.allclose(rh, rh2, atol=1e-4) and torch.allclose(rw, rw2, atol=1e-4)
    drh, drw = torch.randn_like(rh), torch.randn_like(rw)
    dq, dRh, dRw = eng._rel_bwd(q, Rh, Rw, drh, drw)
    dq2, dRh2, dRw2 = vt.relpos_bwd_ref(q, Rh, Rw, drh, drw)
    for a, b in ((dq, dq2), (dRh, dRh2), (dRw, dRw2)):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-4)
