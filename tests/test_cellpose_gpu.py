"""HIP Cellpose post-processing vs the CPU oracle (bioengine_worker_amd/cellpose/reference.py)."""
import numpy as np
import pytest
import torch

from bioengine_worker_amd.cellpose import reference as ref
from tests.test_cellpose_reference import disk_labels, flows_from_labels


def _match_fraction(a, b):
    """Fraction of foreground pixels whose label agrees after optimal one-to-one relabelling of b."""
    agree = 0
    for lab in np.unique(a[a > 0]):
        vals, counts = np.unique(b[a == lab], return_counts=True)
        agree += counts[vals > 0].max() if (vals > 0).any() else 0
    return agree / max(1, (a > 0).sum())


@pytest.mark.gpu
def test_masks_to_flows_gpu_matches_reference(gpu):
    from bioengine_worker_amd.cellpose.gpu import masks_to_flows_gpu

    Ms = [disk_labels(96, 128, 8, seed=s) for s in range(3)]
    M = torch.from_numpy(np.stack(Ms)).to(gpu)
    mu, _, _ = masks_to_flows_gpu(M)
    for b in range(3):
        mref = ref.masks_to_flows(Ms[b])
        err = np.abs(mu[b].cpu().numpy() - mref).max()
        assert err < 2e-3, err


@pytest.mark.gpu
def test_masks_to_flows_every_lds_bucket(gpu):
    """One mask per LDS bucket of the one-workgroup path (64/128/256/512-thread blocks, up to
    ~95 x 95 boxes in a single CU's LDS), each against the numpy oracle."""
    from bioengine_worker_amd.cellpose import gpu as cg

    M = np.zeros((1, 260, 260), np.int32)
    yy, xx = np.mgrid[0:260, 0:260]
    for lab, (cy, cx, r) in enumerate([(12, 12, 8), (40, 40, 12), (80, 30, 17), (40, 100, 24), (130, 60, 30),
                                       (160, 180, 44)], start=1):
        # off-grid centres: no mirror symmetry, so no exact-zero gradient ties between fp orders
        M[0][(yy - cy - 0.37) ** 2 + ((xx - cx - 0.21) * 1.1) ** 2 < r * r] = lab
    w = cg._diffuse_lds_bytes(torch.tensor([90]), torch.tensor([80]))
    assert int(w) <= cg.LDS_DIFFUSE_BYTES
    mu, _, _ = cg.masks_to_flows_gpu(torch.from_numpy(M).to(gpu))
    mref = ref.masks_to_flows(M[0])
    assert np.abs(mu[0].cpu().numpy() - mref).max() < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["tiled", "block"])
def test_big_mask_global_scratch_path(gpu, mode, monkeypatch):
    from bioengine_worker_amd.cellpose import gpu as cg

    monkeypatch.setattr(cg, "BIG_MASK_MODE", mode)
    M = np.zeros((2, 200, 220), np.int32)
    M[0, 10:190, 10:210] = 1  # box exceeds the LDS budget -> big-mask path
    M[0, 50:60, 50:60] = 2
    yy, xx = np.mgrid[0:200, 0:220]
    M[1][((yy - 100) ** 2 / 90 ** 2 + (xx - 120) ** 2 / 70 ** 2) < 1] = 1  # ellipse, ragged tile edges
    M[1, 5:20, 5:200] = 2
    M[1, 20:24, 30:40] = 2  # break the strip's symmetry (its centre flow is otherwise a rounding tie)
    mu, _, _ = cg.masks_to_flows_gpu(torch.from_numpy(M).to(gpu))
    for b in range(2):
        mref = ref.masks_to_flows(M[b])
        assert np.abs(mu[b].cpu().numpy() - mref).max() < 2e-3, b


@pytest.mark.gpu
def test_compute_masks_gpu_matches_reference(gpu):
    from bioengine_worker_amd.cellpose.gpu import compute_masks_gpu

    ys, refs = [], []
    for s in range(4):
        M = disk_labels(128, 160, 10, seed=10 + s)
        dP, cp = flows_from_labels(M)
        ys.append(np.concatenate([dP, cp[None]], 0))
        refs.append(ref.compute_masks(dP, cp))
    y = torch.from_numpy(np.stack(ys)).to(gpu)
    out = compute_masks_gpu(y).cpu().numpy()
    for b in range(4):
        assert out[b].max() == refs[b].max()
        assert _match_fraction(refs[b], out[b]) > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1])
def test_plan_masks_kernel_matches_torch_planner(gpu, kind):
    """be_cp_plan_masks (one launch) vs the torch planner it replaces: same jobs per bucket (order
    inside a bucket is free), same scratch total, same per-image iteration counts."""
    from bioengine_worker_amd.cellpose import gpu as cg

    g = torch.Generator().manual_seed(3)
    B, H, W = 3, 200, 180
    M = torch.zeros(B, H, W, dtype=torch.int32)
    for b in range(B):
        lab = 0
        for _ in range(40):
            h, w = int(torch.randint(2, 40, (1,), generator=g)), int(torch.randint(2, 40, (1,), generator=g))
            y, x = int(torch.randint(0, H - h, (1,), generator=g)), int(torch.randint(0, W - w, (1,), generator=g))
            lab += 1
            M[b, y:y + h, x:x + w] = lab
        M[b, 5:170, 3:150][M[b, 5:170, 3:150] == 0] = lab + 1  # one mask bigger than any LDS bucket
    M = M.to(gpu)
    nlab = int(M.max()) + 1
    bbox = cg.mask_bboxes(M, nlab)
    if kind == 0:
        caps, lds, scr, valid = [c for c, _ in cg.DIFFUSE_BUCKETS], cg._diffuse_lds_bytes, cg._diffuse_scratch_doubles, None
    else:
        caps, lds, scr = [cg.LDS_FILL_BYTES], (lambda ly, lx: (ly + 2) * (lx + 2)), (lambda ly, lx: (ly + 2) * (lx + 2))
        valid = torch.rand(B, nlab, generator=g).to(gpu) > 0.3
    got, tot, niter = cg._plan_masks(bbox, valid, kind, caps)
    present = bbox[..., 1] >= 0
    present[:, 0] = False
    keep = present if valid is None else present & valid
    ar = torch.arange(B * nlab, device=gpu)
    want, wtot = cg._plan_jobs(bbox.view(-1, 4), (ar // nlab).int(), (ar % nlab).int(), lds, caps, scr,
                               valid=keep.view(-1))
    assert sum(int(x.shape[0]) for x in got) == int(keep.sum())
    assert kind == 1 or got[-1].shape[0] >= 1  # the diffusion plan has a beyond-LDS mask
    for a, b in zip(got, want):
        ka = sorted(map(tuple, a[:, :3].tolist()))
        kb = sorted(map(tuple, b[:, :3].tolist()))
        assert ka == kb
    assert tot == wtot
    big = got[-1][:, 3].tolist()
    assert len(set(big)) == len(big) and all(x >= 0 for x in big) and all(x == -1 for x in got[0][:, 3].tolist())
    if kind == 0:
        ext = (bbox[..., 1] - bbox[..., 0] + bbox[..., 3] - bbox[..., 2] + 4).clamp(min=0) * present
        assert torch.equal(niter, (2 * ext.max(dim=1).values).int())


@pytest.mark.gpu
def test_fill_holes_gpu(gpu):
    from bioengine_worker_amd.cellpose.gpu import fill_holes_gpu

    M = np.zeros((64, 64), np.int32)
    M[5:30, 5:30] = 3
    M[10:14, 10:14] = 0
    M[40:42, 40:42] = 5
    M[40:60, 10:30] = 7
    out = fill_holes_gpu(torch.from_numpy(M[None]).to(gpu), min_size=15)[0].cpu().numpy()
    np.testing.assert_array_equal(out, ref.fill_holes_and_remove_small_masks(M, 15))


@pytest.mark.gpu
def test_fill_holes_wave_kernel_matches_lds_kernel_and_oracle(gpu, monkeypatch):
    """One-wave bit-row hole filling (boxes + ring <= 64 x 64, and <= 256 x 128) vs the LDS
    flood-fill kernel and the numpy oracle, on rings, nested labels, boxes at the size limits of
    each kernel, multi-slot rows, islands and random blobs."""
    from bioengine_worker_amd.cellpose import gpu as cg

    rng = np.random.default_rng(7)
    M = np.zeros((2, 200, 240), np.int32)
    yy, xx = np.mgrid[0:200, 0:240]
    M[0][((yy - 40) ** 2 + (xx - 40) ** 2 < 30 ** 2) & ((yy - 40) ** 2 + (xx - 40) ** 2 >= 12 ** 2)] = 1  # ring, 61 px box
    M[0][(yy - 40) ** 2 + (xx - 40) ** 2 < 4 ** 2] = 2  # another label inside the hole
    M[0, 100:162, 5:67] = 3  # 62 x 62 box: the largest one-wave box
    M[0, 110:150, 15:55] = 0  # its hole
    M[0, 120:125, 30:35] = 4
    M[0, 100:163, 100:110] = 5  # 63 rows (65 with the ring): the 256 x 128 bit-row kernel
    M[0, 120:130, 103:107] = 0
    M[0, 30:160, 205:235] = 8  # 130 rows: three row slots per lane
    M[0, 40:150, 210:230] = 0
    M[0, 60:70, 215:220] = 8   # an island inside its own hole
    M[0, 170:198, 5:235] = 9   # 230 columns: the LDS kernel
    M[0, 175:190, 10:200] = 0
    M[0, 10:20, 150:230] = 6
    M[0, 12:18, 152:160] = 0
    M[0, 14:16, 170:200] = 0
    lab = 7
    for _ in range(60):  # random blobs with holes
        cy, cx, r = rng.integers(10, 190), rng.integers(10, 230), rng.integers(3, 12)
        blob = ((yy - cy) ** 2 + (xx - cx) ** 2 < r * r) & (rng.random((200, 240)) > 0.15)
        M[1][blob] = lab
        lab += 1
    Mt = torch.from_numpy(M).to(gpu)
    monkeypatch.setattr(cg, "FILL_WAVE", False)
    lds = cg.fill_holes_gpu(Mt, min_size=15).cpu().numpy()
    monkeypatch.setattr(cg, "FILL_WAVE", True)
    wave = cg.fill_holes_gpu(Mt, min_size=15).cpu().numpy()
    np.testing.assert_array_equal(wave, lds)
    for b in range(2):
        np.testing.assert_array_equal(wave[b], ref.fill_holes_and_remove_small_masks(M[b], 15))


@pytest.mark.gpu
def test_tiles_gather_blend_roundtrip(gpu):
    from bioengine_worker_amd.cellpose.gpu import TilePlan

    x = torch.randn(2, 2, 300, 260, device=gpu)
    plan = TilePlan(300, 260, device=gpu)
    t = plan.gather(x, 8)
    assert t.shape == (2 * plan.nt, plan.by, plan.bx, 8)
    yt = t[..., :2].permute(0, 3, 1, 2).float().contiguous()
    back = plan.blend(yt, 2)
    assert ((back - x).abs() <= 8e-3 * x.abs() + 1e-3).all()  # bf16 rounding only


@pytest.mark.gpu
def test_runner_end_to_end(gpu):
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, synthetic_cells

    imgs = synthetic_cells(2, 256, 256, ncells=30)
    r = CellposeRunner(device=gpu)
    masks, flows, styles = r.eval(imgs)
    assert masks.shape == (2, 256, 256) and flows.shape == (2, 3, 256, 256) and styles.shape == (2, 256)
    assert torch.isfinite(flows).all()


@pytest.mark.gpu
def test_follow_flows_launch_variants_identical(gpu, monkeypatch):
    """The XCD-ordered, block-compacted flow-following launches (256-pixel blocks, and 1,024 pooled) give bit-identical masks to the plain
    pixel-per-lane launch (same per-pixel float sequence, order-independent histogram atomics)."""
    from bioengine_worker_amd.cellpose import gpu as cg

    ys = []
    for s in range(3):
        M = disk_labels(128, 160, 10, seed=40 + s)
        dP, cp = flows_from_labels(M)
        ys.append(np.concatenate([dP, cp[None]], 0))
    y = torch.from_numpy(np.stack(ys)).to(gpu)
    outs = []
    for entry in ("be_cp_follow_flows", "be_cp_follow_flows_xcd", "be_cp_follow_flows_xcd_pool", "be_cp_follow_flows_lds",
                  "be_cp_follow_flows_lds:32"):
        name, _, tile = entry.partition(":")
        monkeypatch.setattr(cg, "FOLLOW_FLOWS_ENTRY", name)
        monkeypatch.setenv("BE_FOLLOW_TILE", tile or "0")
        outs.append(cg.compute_masks_gpu(y).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.gpu
@pytest.mark.parametrize("shape,kind", [((3, 2, 37, 53), "float"), ((4, 2, 128, 128), "uint16"),
                                        ((2, 1, 64, 64), "const"), ((32, 2, 512, 512), "uint16"),
                                        ((2, 3, 100, 101), "neg")])
def test_normalize99_radix_select_matches_sort_and_numpy(gpu, shape, kind):
    """HIP radix-select percentile normalisation == the sort formulation == np.percentile oracle."""
    from bioengine_worker_amd.cellpose.gpu import normalize99, normalize99_sort

    g = torch.Generator().manual_seed(0)
    if kind == "uint16":  # microscopy-like: many ties, a dominant background mode
        x = (torch.rand(shape, generator=g) ** 4 * 4000).round()
    elif kind == "const":
        x = torch.full(shape, 7.0)
        x[1] = torch.rand(shape[1:], generator=g)
    elif kind == "neg":
        x = torch.randn(shape, generator=g) * 100
    else:
        x = torch.rand(shape, generator=g)
    xd = x.to(gpu)
    a = normalize99(xd)
    b = normalize99_sort(xd)
    torch.testing.assert_close(a, b, rtol=0, atol=1e-6)
    if kind != "const":
        xn = x[0, 0].numpy().astype(np.float64)
        p1, p99 = np.percentile(xn, 1), np.percentile(xn, 99)
        np.testing.assert_allclose(a[0, 0].cpu().numpy(), (xn - p1) / (p99 - p1), rtol=1e-4, atol=1e-4)
    normalize99(xd)  # second call reuses the (self-clearing) workspace
    torch.testing.assert_close(normalize99(xd), b, rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_sparse_diffusion_bit_identical_to_dense(gpu, monkeypatch):
    """The sparse pixel-list sweep (thin / irregular masks) and the compact work-queue kernel
    (diffuse_q_kernel, the default) give exactly the dense sweep's flows: same sums in the same
    order, centre source folded into the reads."""
    import os

    from bioengine_worker_amd.cellpose import gpu as cg

    rng = np.random.default_rng(5)
    M = np.zeros((2, 200, 220), np.int32)
    lab = 0
    for b in range(2):
        for _ in range(40):  # random walks: thin, branching, low box fill
            lab += 1
            y, x = rng.integers(10, 190), rng.integers(10, 210)
            for _ in range(rng.integers(20, 160)):
                M[b, y, x] = lab
                y = int(np.clip(y + rng.integers(-1, 2), 1, 198))
                x = int(np.clip(x + rng.integers(-1, 2), 1, 218))
    M[1, 150:180, 5:35] = lab + 1  # a 900-pixel blob: a workgroup job of the queue kernel
    Mt = torch.from_numpy(M).to(gpu)
    old = os.environ.get("BE_DIFFUSE_VARIANT")
    try:
        monkeypatch.setattr(cg, "DIFFUSE_QUEUE", False)
        os.environ["BE_DIFFUSE_VARIANT"] = "3"
        dense, _, _ = cg.masks_to_flows_gpu(Mt)
        os.environ["BE_DIFFUSE_VARIANT"] = "0"
        sparse, _, _ = cg.masks_to_flows_gpu(Mt)
        monkeypatch.setattr(cg, "DIFFUSE_QUEUE", True)
        queued, _, _ = cg.masks_to_flows_gpu(Mt)
    finally:
        if old is None:
            os.environ.pop("BE_DIFFUSE_VARIANT", None)
        else:
            os.environ["BE_DIFFUSE_VARIANT"] = old
    torch.cuda.synchronize()
    assert dense.abs().sum() > 0
    assert torch.equal(dense, sparse)
    assert torch.equal(dense, queued)


@pytest.mark.gpu
def test_diffusion_queue_plan_buckets(gpu):
    """Plan kind 2: masks of <= 256 pixels (box width + 2 <= 256) are wave jobs, <= 2048 pixels
    (the default 512-thread build; 1024 in the 256-thread one) workgroup jobs, the rest keep kind
    0's buckets; every present mask lands in exactly one."""
    from bioengine_worker_amd.cellpose import gpu as cg

    M = torch.zeros(2, 300, 320, dtype=torch.int32)
    M[0, 5:15, 5:20] = 1      # 150 px: wave
    M[0, 20:50, 5:35] = 2     # 900 px: workgroup
    M[0, 70:290, 5:300] = 3   # 64900 px: kind-0 buckets
    M[1, 5:6, 2:300] = 1      # 298 px thin line: workgroup (pixels > 256)
    M[1, 10:11, 2:4] = 2      # 2 px: wave
    M = M.to(gpu)
    nlab = 4
    counts = cg.label_counts(M, nlab)
    bbox = cg.mask_bboxes(M, nlab)
    got, _, _ = cg._plan_finish([cg._plan_launch(bbox, None, 2, cg.DIFFUSE_CAPS, counts)])[0]
    assert len(got) == len(cg.DIFFUSE_BUCKETS) + 4
    key = lambda t: sorted((int(r[0]) & 0xFFFFFFFF, int(r[0]) >> 32) for r in t.cpu())
    assert key(got[0]) == [(0, 1), (1, 2)]
    assert key(got[1]) == [(0, 2), (1, 1)]
    assert sum(len(key(g)) for g in got[2:]) == 1


@pytest.mark.gpu
def test_cross_batch_stream_and_locked_eval_match_eval(gpu):
    """CellposeRunner.stream (net of batch i+1 over masks of batch i on a second stream) and
    eval_locked from two threads (the served path) give eval()'s masks and flows.  eval() itself is
    not bitwise repeatable: the style reduction's float atomics move style by ~1e-8, which flips a
    few bf16 roundings downstream (two eval() calls of the same batch differ by up to ~0.04 in single
    flow pixels, tools/debug_stream.py) -- so flows are compared by relative RMS."""
    import threading

    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, synthetic_cells

    r = CellposeRunner(device=gpu, seed=1)
    batches = [torch.from_numpy(synthetic_cells(3, 256, 256, ncells=25, seed=s)).to(gpu) for s in range(4)]
    ref_out = [r.eval(b) for b in batches]
    st = r.stream()
    got = [st.submit(b) for b in batches] + [st.flush()]
    assert got[0] is None
    def same(m, f, mr, fr):
        rel = ((f - fr).norm() / fr.norm()).item()
        assert rel < 2e-3, rel
        assert (m != mr).float().mean().item() < 1e-3

    for (m, f, s), (mr, fr, sr) in zip(got[1:], ref_out):
        same(m, f, mr, fr)
    net_lock, mask_lock = threading.Lock(), threading.Lock()
    res = [None] * len(batches)

    def work(i):
        m, f, _, ev = r.eval_locked(batches[i], net_lock, mask_lock)
        ev.synchronize()
        # m lives in the mask stream's pool; the clones run on this thread's stream, queued behind
        # other threads' network kernels: without record_stream, m's block could be handed to the
        # next batch's mask stage before the clone has read it (a rare failure of this test)
        cur = torch.cuda.current_stream()
        m.record_stream(cur)
        f.record_stream(cur)
        res[i] = (m.clone(), f.clone())

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(batches))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    for (m, f), (mr, fr, _) in zip(res, ref_out):
        same(m, f, mr, fr)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 3])
def test_graphed_network_stage_identical_to_eager(gpu, B):
    """Small batches replay normalize99 + tiling + CPnet + blend from a HIP graph per shape: the
    flows, styles and masks equal the eager run's bit for bit, also on a second replay with new input."""
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells

    runner = CellposeRunner(device=gpu, seed=0)
    p = EvalParams(niter=200, flow_threshold=0.4, min_size=15)
    for seed in (0, 1):
        imgs = torch.from_numpy(synthetic_cells(B, 512, 512, nchan=2, seed=seed)).to(gpu)
        runner.GRAPH_NET_MAX_B = 8
        mg, fg, sg = runner.eval(imgs, p)
        runner.GRAPH_NET_MAX_B = 0
        me, fe, se = runner.eval(imgs, p)
        assert torch.equal(fg, fe) and torch.equal(sg, se) and torch.equal(mg, me)
    assert any(v for v in runner._net_graphs.values())  # the graph path actually ran
