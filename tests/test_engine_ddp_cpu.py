"""Data-parallel CPnet training through the hand-written engine on gloo (2 ranks): gradient buckets
are released by the engine's explicit readiness calls (no autograd hooks), the all-reduced gradient
equals the mean of the per-rank engine gradients, and both ranks end the AdamW step bit-identical."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _batch(rank, B=2, S=32):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(B, 2, S, S, generator=g)
    lbl = torch.zeros(B, 3, S, S)
    lbl[:, 0] = (torch.rand(B, S, S, generator=g) > 0.6).float()
    lbl[:, 1:] = 0.3 * torch.randn(B, 2, S, S, generator=g)
    return x, lbl


def _net():
    from bioengine_worker_amd.models.cpnet import CPnet

    return CPnet(nbase=(2, 8, 16, 16, 32)).randomize_(0).train()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bioengine_worker_amd.ops import train_ops
    from bioengine_worker_amd.parallel.ddp import BucketedAllReduce, FlatParams
    from bioengine_worker_amd.train.cpnet_engine import CPnetTrainEngine

    net = _net()
    fp = FlatParams(net, "cpu")
    ar = BucketedAllReduce(fp, bucket_mb=0.01)  # several buckets
    eng = CPnetTrainEngine(net, fp, B=2, S=32, device="cpu")
    x, lbl = _batch(rank)
    eng.loss_and_backward(x, lbl, on_params_ready=ar.mark_ready)
    scale = ar.finish()
    g = (fp.grad * scale).clone()
    m, v = torch.zeros_like(fp.flat), torch.zeros_like(fp.flat)
    train_ops.adamw_flat_(fp.flat, fp.grad, m, v, lr=1e-3, step=1, weight_decay=1e-4, grad_scale=scale)
    # numpy copies travel by value (a torch tensor would be shared through a shm file that vanishes
    # when this process exits before the parent reads it)
    q.put((rank, g.numpy().copy(), fp.flat.numpy().copy(), len(ar.buckets)))
    dist.destroy_process_group()


@pytest.mark.unit
def test_engine_ddp_matches_mean_of_rank_grads():
    world = 2
    port = 29700 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
    from bioengine_worker_amd.parallel.ddp import FlatParams
    from bioengine_worker_amd.train.cpnet_engine import CPnetTrainEngine

    grads = []
    for r in range(world):
        net = _net()
        fp = FlatParams(net, "cpu")
        eng = CPnetTrainEngine(net, fp, B=2, S=32, device="cpu")
        eng.loss_and_backward(*_batch(r))
        grads.append(fp.grad.clone())
    mean = sum(grads) / world
    for rank, g, flat, nb in res:
        assert nb > 1
        torch.testing.assert_close(torch.from_numpy(g), mean, rtol=1e-5, atol=1e-7)
    assert (res[0][2] == res[1][2]).all()
