"""ZeRO-1 data-parallel AdamW (parallel/ddp.py ShardedAdamW) against the bucketed all-reduce path:
after 3 steps on gloo at world 2 and 3, every rank's parameters and (synced) AdamW moments equal the
all-reduce + full-AdamW result."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bioengine_worker_amd.ops import train_ops
from bioengine_worker_amd.parallel.ddp import BucketedAllReduce, FlatParams, ShardedAdamW


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(37, 53), torch.nn.ReLU(), torch.nn.Linear(53, 29), torch.nn.Tanh(),
                               torch.nn.Linear(29, 11))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ref, zer = _net(), _net()
        fa = FlatParams(ref, "cpu")
        fz = FlatParams(zer, "cpu", bucket_mb=0.001, bucket_multiple=4 * world)  # ~260 elements: 3 buckets
        ar = BucketedAllReduce(fa, bucket_mb=0.001)
        ma, va = torch.zeros_like(fa.flat), torch.zeros_like(fa.flat)
        mz, vz = torch.zeros_like(fz.flat), torch.zeros_like(fz.flat)
        zo = ShardedAdamW(fz, mz, vz)
        assert len(zo.buckets) >= 3
        g = torch.Generator().manual_seed(100 + rank)  # every rank sees different data
        for step in range(1, 4):
            x = torch.randn(8, 37, generator=g)
            y = torch.randn(8, 11, generator=g)
            for net, fp in ((ref, fa), (zer, fz)):
                fp.zero_grad()
                torch.nn.functional.mse_loss(net(x), y).backward()
            scale = ar.finish()
            train_ops.adamw_flat_(fa.flat, fa.grad, ma, va, lr=1e-2, step=step, weight_decay=0.1, grad_scale=scale)
            zo.step(lr=1e-2, step=step, weight_decay=0.1)
        zo.sync_moments()
        # the padded layouts differ: compare parameter by parameter
        errs = []
        for pa, pz in zip(fa.params, fz.params):
            errs.append((pa - pz).abs().max().item())
        for (oa, oz, p) in zip(fa.offsets, fz.offsets, fa.params):
            k = p.numel()
            errs.append((ma[oa:oa + k] - mz[oz:oz + k]).abs().max().item())
            errs.append((va[oa:oa + k] - vz[oz:oz + k]).abs().max().item())
        q.put((rank, max(errs), fz.flat.clone()))
    except Exception as e:  # noqa: BLE001 -- report instead of leaving the parent waiting
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_adamw_matches_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29610 + world
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, err, _ in res:
        assert not isinstance(err, str), (rank, err)
        assert err < 1e-6, (rank, err)
    flats = [r[2] for r in sorted(res, key=lambda r: r[0])]
    for f in flats[1:]:
        assert torch.equal(f, flats[0])  # every rank holds the same gathered parameters


def test_bucket_layout_padding():
    from bioengine_worker_amd.parallel.ddp import bucket_bounds

    offs, bks = bucket_bounds([5, 7, 300, 2, 9], cap=16, multiple=12)
    assert offs[0] == 0 and offs[1] == 8
    assert all((e - s) % 12 == 0 for s, e, _ in bks)
    assert [m for _, _, m in bks] == [[0, 1], [2], [3, 4]]  # a bucket closes once it reaches the cap
    assert bks[0][1] == 24 and offs[2] == 24                   # 16 elements padded to 24
    assert bks[2][0] == bks[1][1] and offs[3] == bks[2][0]
