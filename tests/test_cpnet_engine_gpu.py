"""HIP training kernels (csrc/kernels/conv_train.hip) against their PyTorch fp32 references, and the
whole hand-written CPnet training step against fp32 autograd on the GPU."""
import copy

import pytest
import torch

from bioengine_worker_amd.ops import conv_train as ct

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


@pytest.mark.parametrize("ks,cin,cin_valid,cy,cout_valid,inmode,use_x2,H", [
    (3, 32, 32, 64, 64, "none", False, 64),
    (3, 32, 32, 32, 32, "pool2", False, 32),
    (3, 64, 64, 32, 32, "up2", False, 64),
    (3, 32, 32, 32, 32, "none", True, 48),
    (3, 8, 2, 32, 32, "none", False, 40),
    (1, 8, 2, 32, 32, "none", False, 32),
    (1, 32, 32, 8, 3, "none", False, 64),
    (1, 256, 256, 128, 128, "up2", False, 16),
])
def test_wgrad_kernel(gpu, ks, cin, cin_valid, cy, cout_valid, inmode, use_x2, H):
    torch.manual_seed(0)
    N = 3
    Hs = H * 2 if inmode == "pool2" else (H // 2 if inmode == "up2" else H)
    x = torch.randn(N, Hs, Hs, cin, device=gpu).to(torch.bfloat16)
    if cin_valid < cin:
        x[..., cin_valid:] = 0
    x2 = torch.randn(N, H, H, cin, device=gpu).to(torch.bfloat16) if use_x2 else None
    scale = (1 + 0.2 * torch.randn(cin, device=gpu)).float()
    shift = (0.3 * torch.randn(N, cin, device=gpu)).float()
    dy = torch.randn(N, H, H, cy, device=gpu).to(torch.bfloat16)
    dw = torch.zeros(cout_valid, cin_valid, ks, ks, device=gpu)
    db = torch.zeros(cout_valid, device=gpu)
    ct.conv_wgrad(x, dy, ks=ks, cin_valid=cin_valid, cout_valid=cout_valid, dw=dw, db=db, inmode=inmode, x2=x2,
                  scale=scale, shift=shift, relu=True)
    dw_ref = torch.empty(cout_valid, cin_valid, ks, ks)
    db_ref = torch.empty(cout_valid)
    # CPU reference on the same bf16 inputs; activation rounded to bf16 like the kernel's LDS staging
    from bioengine_worker_amd.ops.conv import _act_ref

    a = _act_ref(x.cpu().float(), None if x2 is None else x2.cpu().float(), scale.cpu(), shift.cpu(), True, inmode)
    a = a.to(torch.bfloat16).float()[:, :cin_valid]
    g = dy.cpu().float()[..., :cout_valid].permute(0, 3, 1, 2)
    dw_ref = torch.nn.grad.conv2d_weight(a, (cout_valid, cin_valid, ks, ks), g, padding=ks // 2)
    db_ref = g.sum((0, 2, 3))
    torch.cuda.synchronize()
    assert _rel(dw.cpu(), dw_ref) < 2e-3
    assert _rel(db.cpu(), db_ref) < 2e-3


def _site(dev, N, C, c_valid, nunits, relus, groups=0):
    units = []
    for k in range(nunits):
        units.append(ct.BnUnit(gamma=(1 + 0.1 * torch.randn(c_valid)).to(dev), beta=(0.1 * torch.randn(c_valid)).to(dev),
                               run_mean=None if groups else torch.zeros(c_valid, device=dev),
                               run_var=None if groups else torch.ones(c_valid, device=dev),
                               relu=relus[k], scale=torch.zeros((N, C) if groups else (C,), device=dev),
                               shift=torch.zeros(N, C, device=dev),
                               dgamma=torch.zeros(c_valid, device=dev), dbeta=torch.zeros(c_valid, device=dev)))
    stat = torch.zeros(ct.BnSite.stat_numel(N, C, groups), device=dev)
    ticket = torch.zeros(2, dtype=torch.int32, device=dev)
    return ct.BnSite(N, C, c_valid, units, stat, ticket, groups=groups)


def _site_to_cpu(s: ct.BnSite) -> ct.BnSite:
    cpu = lambda t, f: None if t is None else f(t.cpu())  # noqa: E731
    units = [ct.BnUnit(gamma=u.gamma.cpu(), beta=u.beta.cpu(), run_mean=cpu(u.run_mean, torch.zeros_like),
                       run_var=cpu(u.run_var, torch.ones_like), relu=u.relu, scale=torch.zeros_like(u.scale.cpu()),
                       shift=torch.zeros_like(u.shift.cpu()), dgamma=torch.zeros_like(u.dgamma.cpu()),
                       dbeta=torch.zeros_like(u.dbeta.cpu())) for u in s.units]
    return ct.BnSite(s.N, s.C, s.c_valid, units, torch.zeros_like(s.stat.cpu()), torch.zeros(2, dtype=torch.int32),
                     groups=s.groups)


@pytest.mark.parametrize("inmode,use_x2,use_feat,nunits,C,c_valid,groups", [
    ("none", False, False, 1, 32, 32, 0),
    ("pool2", False, False, 2, 64, 64, 0),
    ("up2", False, False, 2, 128, 128, 0),
    ("none", True, True, 1, 32, 32, 0),
    ("none", False, True, 1, 256, 256, 0),
    ("none", False, False, 2, 8, 2, 0),
    # GroupNorm: per-image, per-group statistics (the DP training default)
    ("none", False, False, 1, 32, 32, 8),
    ("pool2", False, False, 2, 64, 64, 8),
    ("up2", True, True, 1, 128, 128, 8),
    ("none", False, True, 1, 256, 256, 8),
    ("none", False, False, 2, 8, 2, 1),
])
def test_bn_site_kernels(gpu, inmode, use_x2, use_feat, nunits, C, c_valid, groups):
    torch.manual_seed(1)
    N, H = 3, 32
    Hs = H * 2 if inmode == "pool2" else (H // 2 if inmode == "up2" else H)
    x = (torch.randn(N, Hs, Hs, C, device=gpu) + 0.5).to(torch.bfloat16)
    if c_valid < C:
        x[..., c_valid:] = 0
    x2 = torch.randn(N, H, H, C, device=gpu).to(torch.bfloat16) if use_x2 else None
    feat = (0.5 * torch.randn(N, C, device=gpu)) if use_feat else None
    relus = [False, True][-nunits:] if nunits == 2 else [True]
    s = _site(gpu, N, C, c_valid, nunits, relus, groups)
    sc = _site_to_cpu(s)
    cpu = lambda t: None if t is None else t.cpu()  # noqa: E731
    s.stats(x, inmode, x2, feat)
    sc.stats(cpu(x), inmode, cpu(x2), cpu(feat))
    for u, v in zip(s.units, sc.units):
        assert _rel(u.scale.cpu(), v.scale) < 1e-4
        assert _rel(u.shift.cpu(), v.shift) < 1e-4
        if not groups:
            assert _rel(u.run_var.cpu(), v.run_var) < 1e-4
    dacts = [torch.randn(N, H, H, C, device=gpu).to(torch.bfloat16) for _ in range(nunits)]
    dfeat = torch.zeros(N, C, device=gpu) if use_feat else None
    dfeat_c = torch.zeros(N, C) if use_feat else None
    s.bwd_reduce(x, dacts, inmode, x2, feat, dfeat)
    sc.bwd_reduce(cpu(x), [cpu(d) for d in dacts], inmode, cpu(x2), cpu(feat), dfeat_c)
    for u, v in zip(s.units, sc.units):
        assert _rel(u.dgamma.cpu(), v.dgamma) < 2e-3
        assert _rel(u.dbeta.cpu(), v.dbeta) < 2e-3
    if use_feat:
        assert _rel(dfeat.cpu(), dfeat_c) < 2e-3
    dx = torch.randn(N, Hs, Hs, C, device=gpu).to(torch.bfloat16)
    dx_c = dx.cpu().float().clone()
    dx2 = torch.zeros(N, H, H, C, device=gpu, dtype=torch.bfloat16) if use_x2 else None
    dx2_c = torch.zeros(N, H, H, C) if use_x2 else None
    s.bwd_apply(x, dacts, inmode, x2, feat, dx=dx, dx_acc=True, dx2=dx2, dx2_acc=False)
    sc.bwd_apply(cpu(x), [cpu(d) for d in dacts], inmode, cpu(x2), cpu(feat), dx=dx_c, dx_acc=True, dx2=dx2_c)
    torch.cuda.synchronize()
    assert _rel(dx.cpu(), dx_c) < 2e-2  # bf16 storage of the accumulated gradient
    if use_x2:
        assert _rel(dx2.cpu(), dx2_c) < 2e-2


def test_pack_weights_kernel(gpu):
    from bioengine_worker_amd.ops.conv import PackedConv

    w = torch.randn(64, 32, 3, 3)
    flat = torch.cat([torch.zeros(4), w.reshape(-1)]).to(gpu)
    pc = PackedConv.from_weight(w)
    wt = w.flip(2, 3).transpose(0, 1).contiguous()
    pct = PackedConv.from_weight(wt)
    n0 = pc.wp.numel()
    n1 = pct.wp.numel()
    descs = torch.tensor([[4, 0, 64, 32, 3, pc.cout_pad, pc.cin_pad, pc.ck, pc.kp, 0],
                          [4, n0, 64, 32, 3, pct.cout_pad, pct.cin_pad, pct.ck, pct.kp, 1]], dtype=torch.int32, device=gpu)
    arena = torch.empty(n0 + n1, dtype=torch.bfloat16, device=gpu)
    ct.pack_weights(descs, 2, max(n0, n1), flat, arena)
    torch.cuda.synchronize()
    assert torch.equal(arena[:n0].cpu().view_as(pc.wp), pc.wp)
    assert torch.equal(arena[n0:].cpu().view_as(pct.wp), pct.wp)


@pytest.mark.parametrize("B,S,norm", [(4, 128, "batch"), (4, 128, "group")])
def test_engine_step_vs_autograd(gpu, B, S, norm):
    """bf16 activations through 40 train-mode BN layers of a random-init net decorrelate gradients from
    fp32 by themselves (torch's own bf16 autocast reaches cos ~0.93 here): the engine must agree with
    fp32 autograd as well as autocast-bf16 autograd does."""
    import statistics

    from bioengine_worker_amd.models.cpnet import CPnet
    from bioengine_worker_amd.ops import train_ops
    from bioengine_worker_amd.parallel.ddp import FlatParams
    from bioengine_worker_amd.train.cpnet_engine import CPnetTrainEngine

    torch.manual_seed(0)
    net = CPnet(norm=norm).randomize_(0).train()
    ref = copy.deepcopy(net).to(gpu)
    amp = copy.deepcopy(net).to(gpu)
    x = torch.randn(B, 2, S, S, device=gpu)
    lbl = torch.zeros(B, 3, S, S, device=gpu)
    lbl[:, 0] = (torch.rand(B, S, S, device=gpu) > 0.6).float()
    lbl[:, 1:] = 0.3 * torch.randn(B, 2, S, S, device=gpu)
    loss_ref = train_ops.seg_loss_ref(ref(x)[0], lbl)
    loss_ref.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y_amp = amp(x)[0]
    train_ops.seg_loss_ref(y_amp.float(), lbl).backward()
    net = net.to(gpu)
    fp = FlatParams(net, gpu)
    eng = CPnetTrainEngine(net, fp, B=B, S=S, device=gpu)
    loss = eng.loss_and_backward(x, lbl)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(loss_ref.detach())) < 2e-2 * abs(float(loss_ref.detach())) + 1e-3
    nr, na = dict(ref.named_parameters()), dict(amp.named_parameters())
    gmax = max(p.grad.abs().max().item() for p in ref.parameters() if p.grad is not None)
    ce, ca = [], []
    for name, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g_ref = nr[name].grad.float()
        g = p.grad.float()
        assert torch.isfinite(g).all(), name
        if g.numel() < 16:  # the 2-channel input BN: cosine of 2 numbers is noise
            continue
        if g_ref.abs().max().item() < 1e-3 * gmax:  # conv biases cancelled by the next train-mode BN
            assert g.abs().max().item() < 2e-2 * gmax, name
            continue
        cos = lambda a, b: torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()  # noqa: E731
        ce.append(cos(g, g_ref))
        ca.append(cos(na[name].grad.float(), g_ref))
    assert statistics.median(ce) > statistics.median(ca) - 0.03, (statistics.median(ce), statistics.median(ca))
    assert min(ce) > min(ca) - 0.15, (min(ce), min(ca))


def test_groupnorm_net_inference(gpu):
    """A GroupNorm CPnet (what data-parallel fine-tuning produces) serves through the runner: HIP GN
    statistics + fused convs per tile batch vs the fp32 module on CPU."""
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells
    from bioengine_worker_amd.models.cpnet import CPnet

    net = CPnet(norm="group").randomize_(2)
    img = synthetic_cells(2, 256, 256, ncells=30, seed=1)
    _, yg, sg = CellposeRunner(net=net, device=gpu).eval(img, EvalParams(compute_masks=False))
    _, yc, sc = CellposeRunner(net=net, device="cpu").eval(img, EvalParams(compute_masks=False))
    assert _rel(yg.cpu(), yc) < 5e-2
    assert _rel(sg.cpu(), sc) < 5e-2
