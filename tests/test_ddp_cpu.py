"""Data-parallel bucketed all-reduce on gloo (2 ranks) == single-process gradient on the union batch."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bioengine_worker_amd.parallel.ddp import BucketedAllReduce, FlatParams


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 8))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = _net()
    fp = FlatParams(net)
    ar = BucketedAllReduce(fp, bucket_mb=0.0005)  # force several buckets
    torch.manual_seed(1)
    x = torch.randn(8, 16)
    mine = x[rank::world]
    fp.zero_grad()
    net(mine).pow(2).mean().backward()
    scale = ar.finish()
    q.put((rank, (fp.grad * scale).numpy().copy(), len(ar.buckets)))  # by value, not via a shm file
    dist.destroy_process_group()


@pytest.mark.unit
def test_bucketed_allreduce_matches_single_process():
    world = 2
    port = 29500 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    net = _net()
    fp = FlatParams(net)
    torch.manual_seed(1)
    x = torch.randn(8, 16)
    fp.zero_grad()
    # mean of per-rank means == mean over the union when shards are equal size
    loss = 0.5 * (net(x[0::2]).pow(2).mean() + net(x[1::2]).pow(2).mean())
    loss.backward()
    for rank, g, nb in res:
        assert nb > 1
        g = torch.from_numpy(g)
        assert torch.allclose(g, fp.grad, atol=1e-6), (rank, (g - fp.grad).abs().max())
