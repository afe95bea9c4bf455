"""Data-parallel optimizer paths on gloo (2 ranks, CPU):

* per-bucket AdamW (``BucketedAllReduce.finish_each``: each bucket updated right after its own
  all-reduce) gives exactly the weights of one whole-model AdamW after ``finish()``;
* the bf16 gradient wire (``comm_dtype=torch.bfloat16``, half the all-reduce bytes) stays within a
  stated bound of the fp32 wire over 50 steps: max |w_bf16 - w_fp32| <= 2e-3 (lr 1e-3, so <= 2 steps'
  worth of update), relative RMS <= 2e-3 (docs/dp_comm_budget.md)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bioengine_worker_amd.ops import train_ops
from bioengine_worker_amd.parallel.ddp import BucketedAllReduce, FlatParams

STEPS = 50
LR = 1e-3


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 8))


def _train(rank, world, mode):
    net = _net()
    fp = FlatParams(net)
    comm = torch.bfloat16 if mode == "bf16" else None
    ar = BucketedAllReduce(fp, bucket_mb=0.001, comm_dtype=comm)  # several buckets
    m, v = torch.zeros_like(fp.flat), torch.zeros_like(fp.flat)
    g = torch.Generator().manual_seed(123)
    wt = torch.randn(32, 8, generator=g)
    for step in range(1, STEPS + 1):
        x = torch.randn(16, 32, generator=g)
        y = torch.tanh(x @ wt)
        mine = slice(rank * 8, rank * 8 + 8)
        fp.zero_grad()
        (net(x[mine]) - y[mine]).pow(2).mean().backward()
        if mode == "bucket":
            def upd(s, e, sc):
                sl = slice(s, e)
                train_ops.adamw_flat_(fp.flat[sl], fp.grad[sl], m[sl], v[sl], lr=LR, step=step, weight_decay=1e-4,
                                      grad_scale=sc)
            ar.finish_each(upd)
        else:
            sc = ar.finish()
            train_ops.adamw_flat_(fp.flat, fp.grad, m, v, lr=LR, step=step, weight_decay=1e-4, grad_scale=sc)
    return fp.flat.clone(), len(ar.buckets)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for mode in ("fp32", "bucket", "bf16"):
        w, nb = _train(rank, world, mode)
        out[mode] = w.numpy().copy()
        out["nb"] = nb
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.unit
def test_bucket_adamw_and_bf16_wire():
    world = 2
    port = 31000 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
    for r in range(world):
        o = {k: torch.from_numpy(v) if k != "nb" else v for k, v in res[r].items()}
        assert o["nb"] > 2
        # per-bucket updates are the same elementwise math on the same reduced gradients
        assert torch.equal(o["bucket"], o["fp32"]), (o["bucket"] - o["fp32"]).abs().max()
        d = (o["bf16"] - o["fp32"]).abs()
        rel = (d.pow(2).mean().sqrt() / o["fp32"].pow(2).mean().sqrt()).item()
        assert d.max().item() <= 2e-3 and rel <= 2e-3, (d.max().item(), rel)
    # ranks agree bit-exactly (every rank applies the same reduced gradient)
    for k in ("fp32", "bucket", "bf16"):
        assert (res[0][k] == res[1][k]).all()
