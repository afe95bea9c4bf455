"""GPU numerics of the Cellpose-SAM training path: every HIP backward kernel against its fp32 PyTorch
reference, and the whole engine step (forward + backward, stochastic depth on) against fp32 autograd
through the CPSAM module."""
import copy
import math

import pytest
import torch

from bioengine_worker_amd.ops import vit_train as vt

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.fixture(scope="module")
def dev():
    from bioengine_worker_amd.ops import _native

    _native.hip()
    return torch.device("cuda", 0)


# (B, H) = (2, 3): small grids -> the fused dq + dkv launch; (8, 8) / (16, 32): the two-launch path
@pytest.mark.parametrize("N,bias,B,H", [(1024, True, 2, 3), (1056, True, 2, 3), (257, False, 2, 3),
                                        (1024, True, 8, 8), (1056, True, 8, 8), (257, False, 16, 32)])
def test_attn_bwd_matches_reference(dev, N, bias, B, H):
    torch.manual_seed(0)
    D = 64
    qkv = (torch.randn(B, N, 3, H, D, device=dev) * 0.5).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    rh = rw = None
    if bias:
        Hg = N // 32
        rh = torch.randn(B, H, N, Hg, device=dev) * 0.5
        rw = torch.randn(B, H, N, 32, device=dev) * 0.5
    scale = D ** -0.5
    o, lse = vt.attn_fwd(q, k, v, scale, rh, rw)
    do = (torch.randn(B, N, H, D, device=dev) * 0.5).bfloat16()
    dq, dk, dv, drh, drw = vt.attn_bwd(q, k, v, o, do, lse, scale, rh, rw)
    torch.cuda.synchronize()
    c = lambda t: None if t is None else t.cpu()
    o_r, lse_r = vt.attn_fwd(c(q).float(), c(k).float(), c(v).float(), scale, c(rh), c(rw))
    assert _rel(lse.cpu(), lse_r) < 1e-3
    assert _rel(o.cpu(), o_r) < 1e-2, _rel(o.cpu(), o_r)
    dq_r, dk_r, dv_r, drh_r, drw_r = vt.attn_bwd(c(q).float(), c(k).float(), c(v).float(), c(o).float(),
                                                c(do).float(), lse_r, scale, c(rh), c(rw))
    for name, a, r in (("dq", dq, dq_r), ("dk", dk, dk_r), ("dv", dv, dv_r)):
        assert _rel(a.cpu(), r) < 2e-2, (name, _rel(a.cpu(), r))
    if bias:
        assert _rel(drh.cpu(), drh_r) < 2e-2 and _rel(drw.cpu(), drw_r) < 2e-2


def test_layernorm_gelu_cast_kernels(dev):
    torch.manual_seed(1)
    rows, C, Npr = 4 * 300, 1024, 300
    x = torch.randn(rows, C, device=dev).bfloat16()
    y = torch.randn(rows, C, device=dev).bfloat16()
    w = torch.randn(C, device=dev) * 0.3 + 1
    b = torch.randn(C, device=dev) * 0.1
    rs = torch.tensor([1.0, 0.0, 1.0, 1.0], device=dev)
    xo, out, st = vt.ln_fwd(x, w, b, y=y, rs=rs, rpn=Npr)
    xo_r, out_r, st_r = vt.ln_fwd(x.cpu(), w.cpu(), b.cpu(), y=y.cpu(), rs=rs.cpu(), rpn=Npr)
    assert torch.equal(xo.cpu(), xo_r)
    assert _rel(out.cpu(), out_r) < 1e-2 and _rel(st.cpu(), st_r) < 1e-4
    dh = torch.randn(rows, C, device=dev).bfloat16()
    r1 = torch.randn(rows, C, device=dev)
    res = vt.ln_bwd(dh, xo, st, w, r1=r1, s1=rs, rpn=Npr, want_dxb=True, want_col=True)
    ref = vt.ln_bwd(dh.cpu(), xo.cpu(), st.cpu(), w.cpu(), r1=r1.cpu(), s1=rs.cpu(), rpn=Npr, want_dxb=True,
                    want_col=True)
    for a, r in zip(res, ref):
        assert _rel(a.cpu(), r) < 1e-2
    f = torch.randn(rows, 4 * C, device=dev).bfloat16()
    b1 = torch.randn(4 * C, device=dev) * 0.1
    assert _rel(vt.gelu_fwd(f, b1).cpu(), vt.gelu_fwd(f.cpu(), b1.cpu())) < 1e-2
    dg = torch.randn(rows, 4 * C, device=dev).bfloat16()
    df, db = vt.gelu_bwd(dg, f, b1)
    df_r, db_r = vt.gelu_bwd(dg.cpu(), f.cpu(), b1.cpu())
    assert _rel(df.cpu(), df_r) < 1e-2 and _rel(db.cpu(), db_r) < 1e-2
    g32 = torch.randn(rows, C, device=dev)
    yb, col = vt.scale_cast(g32, rs, Npr)
    yb_r, col_r = vt.scale_cast(g32.cpu(), rs.cpu(), Npr)
    assert torch.equal(yb.cpu(), yb_r) and _rel(col.cpu(), col_r) < 1e-5


@pytest.mark.parametrize("side_wgrad,backend", [(False, "lib"), (True, "lib"), (False, "hip"), (False, "auto")])
def test_cpsam_engine_matches_fp32_autograd(dev, side_wgrad, backend, monkeypatch):
    """GEMM backends: the library (default), the in-house kernels, and the per-shape choice.  The
    biases are made non-zero (randomize_ zeroes them, which once hid a bf16-bias misread in the
    in-house epilogues)."""
    from bioengine_worker_amd.models.cpsam import CPSAM
    from bioengine_worker_amd.ops import gemm as gemm_lib
    from bioengine_worker_amd.ops import gemm_auto, gemm_bf16, train_ops
    from bioengine_worker_amd.parallel.ddp import FlatParams
    from bioengine_worker_amd.train import cpsam_engine
    from bioengine_worker_amd.train.cpsam_engine import CPSAMTrainEngine

    monkeypatch.setattr(cpsam_engine, "gemm", {"lib": gemm_lib, "hip": gemm_bf16, "auto": gemm_auto}[backend])
    monkeypatch.delenv("BE_GEMM_AUTO", raising=False)
    torch.manual_seed(0)
    B = 2
    net = CPSAM(dim=256, depth=2, heads=4, bsize=256).randomize_(0)
    gb = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith("bias"):
                p.copy_(torch.randn(p.shape, generator=gb) * 0.1)
    ref = copy.deepcopy(net).to(dev).train()
    x = torch.randn(B, 3, 256, 256, device=dev)
    lbl = torch.zeros(B, 3, 256, 256, device=dev)
    lbl[:, 0] = (torch.rand(B, 256, 256, device=dev) > 0.6).float()
    lbl[:, 1:] = torch.randn(B, 2, 256, 256, device=dev) * 0.3
    keep = torch.tensor([[1.0, 0.0], [1.0, 1.0]], device=dev)
    y_r = ref(x, keep=keep)[0]
    loss_r = train_ops.seg_loss_ref(y_r, lbl)
    loss_r.backward()
    net = net.to(dev)
    fp = FlatParams(net, dev)
    eng = CPSAMTrainEngine(net, fp, B, dev, side_wgrad=side_wgrad)
    loss = eng.loss_and_backward(x, lbl, keep)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(loss_r)) < 2e-2 * abs(float(loss_r))
    refg = dict(ref.named_parameters())
    for name, p in net.named_parameters():
        if p.requires_grad:
            err = _rel(p.grad, refg[name].grad)
            assert err < 2e-2, (name, err)


def test_cpsam_trainer_steps(dev):
    from bioengine_worker_amd.models.cpsam import CPSAM
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    cfg = TrainConfig(batch_size=2, bsize=256, lr=1e-4, weight_decay=1e-4)
    net = CPSAM(dim=256, depth=2, heads=4, bsize=256).randomize_(0)
    tr = build_trainer(cfg, dev, net=net)
    assert tr.engine_kind == "cpsam"
    batch = synthetic_train_batch(2, 256, device=dev)
    losses = [float(tr.step(*batch)) for _ in range(6)]
    assert all(math.isfinite(l) for l in losses)
    assert min(losses[3:]) < losses[0]
    # the bf16 mirror tracks the fp32 master after the fused AdamW
    eng = tr._cpsam_engine(2)
    assert _rel(eng.mirror.float(), tr.fp.flat) < 1e-2
    m = tr.validate(*batch)
    assert math.isfinite(m["loss"])


def test_cpsam_runner_matches_cpu_reference(dev):
    """Cellpose-SAM inference (HIP engine: flash attention + rel-pos, fused LN, MFMA neck conv) through
    the tiled runner vs the same runner on the fp32 PyTorch module on CPU."""
    import numpy as np

    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells
    from bioengine_worker_amd.models.cpsam import CPSAM

    net = CPSAM(dim=256, depth=2, heads=4, bsize=256).randomize_(1)
    img = synthetic_cells(1, 300, 280, nchan=2, ncells=20, seed=2)
    p = EvalParams(compute_masks=False)
    _, yg, _ = CellposeRunner(net=net, device=dev).eval(img, p)
    _, yc, _ = CellposeRunner(net=net, device="cpu").eval(img, EvalParams(compute_masks=False))
    assert yg.shape == (1, 3, 300, 280)
    assert _rel(yg.cpu(), yc) < 3e-2
    masks, _, _ = CellposeRunner(net=net, device=dev).eval(img)
    assert masks.shape == (1, 300, 280) and np.isfinite(yg.cpu().numpy()).all()


@pytest.mark.parametrize("B", [1, 3])
def test_relpos_kernels_match_fp32_oracle(dev, B):
    """relpos.hip (MFMA, hi/lo-split fp32 operands) vs the fp32 einsum oracle: rel_h / rel_w, dq + dq_rel
    written as bf16 into a packed-dqkv q slot, and the gathered rel-pos table gradients."""
    torch.manual_seed(1)
    g, H, c = 32, 4, 64
    N = g * g
    qkv = (torch.randn(B, N, 3, H, c, device=dev) * 0.5).bfloat16()
    q = qkv[:, :, 0]
    ar = torch.arange(g, device=dev)
    idx = (ar[:, None] - ar[None, :] + g - 1).long()
    tab_h, tab_w = torch.randn(2 * g - 1, c, device=dev) * 0.3, torch.randn(2 * g - 1, c, device=dev) * 0.3
    Rh, Rw = tab_h[idx], tab_w[idx]  # get_rel_pos at q == k size (the kernels gather it themselves)
    rh, rw = vt.relpos_fwd(q, tab_h, tab_w)
    rh_r, rw_r = vt.relpos_fwd_ref(q.cpu(), Rh.cpu(), Rw.cpu())
    assert _rel(rh.cpu(), rh_r) < 1e-4 and _rel(rw.cpu(), rw_r) < 1e-4
    drh, drw = torch.randn(B, H, N, g, device=dev), torch.randn(B, H, N, g, device=dev)
    dq = torch.randn(B, N, H, c, device=dev)
    dq0 = dq.clone()
    dqkv = torch.zeros(B, N, 3, H, c, device=dev, dtype=torch.bfloat16)
    gh, gw = torch.full((2 * g - 1, c), 7.0, device=dev), torch.full((2 * g - 1, c), 7.0, device=dev)
    vt.relpos_bwd_(q, tab_h, tab_w, drh, drw, dq, dqkv[:, :, 0], gh, gw, idx)
    torch.cuda.synchronize()
    dq_rel, dRh, dRw = vt.relpos_bwd_ref(q.cpu(), Rh.cpu(), Rw.cpu(), drh.cpu(), drw.cpu())
    assert _rel(dqkv[:, :, 0].float().cpu(), dq0.cpu() + dq_rel) < 1e-2  # bf16 output
    assert dqkv[:, :, 1:].abs().max() == 0  # k / v slots untouched
    for got, dR in ((gh, dRh), (gw, dRw)):
        ref = torch.zeros(2 * g - 1, c).index_add_(0, idx.cpu().reshape(-1), dR.reshape(-1, c))
        assert _rel(got.cpu(), ref) < 1e-4


def test_cpsam_adamw_overlapped_in_graph_matches_flat_update(dev):
    """AdamW per parameter group inside the captured step (side stream, device-resident lr / bias
    corrections) gives the same weights, moments and bf16 mirror as the flat update after it (not
    bitwise: the rel-pos table gradients accumulate with fp32 atomics, and the bias corrections come
    from the host in double instead of powf; a skipped group would show up as a ~1e-2 difference)."""
    from bioengine_worker_amd.models.cpsam import CPSAM
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    trs = []
    for fuse in (False, True):
        cfg = TrainConfig(batch_size=2, bsize=256, lr=1e-4, weight_decay=1e-4, cpsam_overlap_adamw=fuse)
        tr = build_trainer(cfg, dev, net=CPSAM(dim=256, depth=2, heads=4, bsize=256).randomize_(0))
        tr._init_flat = tr.fp.flat.clone()
        batch = synthetic_train_batch(2, 256, device=dev, seed=3)
        for i in range(4):
            tr.set_lr(1e-4 * (i + 1))  # the schedule must reach the in-graph update
            tr.step(*batch)
        torch.cuda.synchronize()
        trs.append(tr)
    a, b = trs
    assert b._adamw_in_graph and not a._adamw_in_graph
    upd = _rel(a.fp.flat, a._init_flat)  # how far 4 steps moved the weights
    assert upd > 1e-3
    # fused vs flat differ only by atomic-order / bias-correction rounding: far below one update
    assert _rel(b.fp.flat, a.fp.flat) < 0.02 * upd, (_rel(b.fp.flat, a.fp.flat), upd)
    assert _rel(b.m, a.m) < 0.05 and _rel(b._cpsam_engine(2).mirror.float(), a._cpsam_engine(2).mirror.float()) < 0.02 * upd + 1e-3


def test_batched_colsums_bf16_partials_and_slab_sums(dev):
    """Deferred (batched) column reductions, bf16 column partials and split-K slab sums vs torch."""
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(512, 1024), (16, 4096), (3, 3072), (64, 192), (8, 8)] * 12  # 60 > one 48-entry launch
    parts = [torch.randn(r, c, generator=g).to(dev) for r, c in shapes]
    outs = [torch.full((c,), float("nan"), device=dev) for _, c in shapes]
    with vt.defer_colsums() as d:
        for p, o in zip(parts, outs):
            vt._colsum(p, o)
        assert len(d.items) == len(shapes)  # nothing launched before the flush
    torch.cuda.synchronize()
    for p, o in zip(parts, outs):
        torch.testing.assert_close(o, p.sum(0), rtol=1e-5, atol=1e-4)
    for rows, C in ((8192, 3072), (1000, 192), (1, 8)):
        x = torch.randn(rows, C, generator=g).to(dev).bfloat16()
        out = torch.empty(C, device=dev)
        vt.colsum_bf16(x, out)
        torch.testing.assert_close(out, x.float().sum(0), rtol=1e-4, atol=1e-2)
    ws = torch.randn(4, 1024, 3072, generator=g).to(dev)
    out = torch.empty(1024, 3072, device=dev)
    vt.sum_slabs(ws, out)
    torch.testing.assert_close(out, ws.sum(0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,k", [(4096, 1024), (1024, 4096), (3072, 1024), (1024, 1024)])
def test_wgrad_split_paths_match_fp32(dev, n, k):
    """Weight-gradient GEMM paths at the batch-8 token count (split-K 2 for the 4096-wide shapes,
    split-K 4 for the <= 192-tile ones, slab sums on the HIP kernel) vs an fp32 matmul."""
    from bioengine_worker_amd.train.cpsam_engine import _wgrad

    g = torch.Generator().manual_seed(11)
    m = 8192
    dy = torch.randn(m, n, generator=g).to(dev).bfloat16()
    x = torch.randn(m, k, generator=g).to(dev).bfloat16()
    out = torch.full((n, k), float("nan"), device=dev)
    _wgrad(dy, x, out)
    ref = dy.float().t() @ x.float()
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-4
