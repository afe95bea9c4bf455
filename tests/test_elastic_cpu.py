"""Elastic data parallelism (parallel/elastic.py) on gloo: 3 ranks train the Cellpose CPnet; member 2
dies mid-run (os._exit right before its step's all-reduce); the survivors detect the failed
collective, agree on the survivor set through the control store, re-init a 2-rank process group,
re-bind the trainer (bucketed all-reduce + weight/moment broadcast) and finish every step with
identical weights."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(member, world, port, q, victim, die_at, n_steps):
    torch.set_num_threads(1)
    from bioengine_worker_amd.parallel.elastic import ElasticWorld, run_elastic
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    ew = ElasticWorld(member, world, master_port=port, backend="gloo", heartbeat_s=0.2, stale_s=1.5,
                      pg_timeout_s=20)
    cfg = TrainConfig(batch_size=1, bsize=64, engine="autograd", graph=False, bucket_mb=2.0)
    tr = build_trainer(cfg, "cpu", world_size=ew.world, rank=ew.rank)
    imgs, lbls = synthetic_train_batch(1, 64, device="cpu", seed=member)
    shrinks = []

    def batches(step, w):
        if member == victim and step == die_at:
            os._exit(17)  # hard failure: no cleanup, sockets just close
        return imgs, lbls

    losses = run_elastic(ew, tr, batches, n_steps, on_shrink=lambda s, m, e: shrinks.append((s, m)))
    q.put((member, losses, shrinks, ew.world, ew.rank, tr.fp.flat.clone(), tr.step_count))
    ew.close()


@pytest.mark.timeout(300)
def test_elastic_shrink_on_rank_failure():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    world, victim, die_at, n_steps = 3, 2, 2, 5
    ps = [ctx.Process(target=_worker, args=(m, world, port, q, victim, die_at, n_steps)) for m in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world - 1):
        m, losses, shrinks, w, r, flat, steps = q.get(timeout=240)
        res[m] = (losses, shrinks, w, r, flat, steps)
    for p in ps:
        p.join(60)
    assert ps[victim].exitcode == 17
    assert sorted(res) == [0, 1]
    for m, (losses, shrinks, w, r, flat, steps) in res.items():
        assert len(losses) == n_steps and all(x == x for x in losses)
        assert shrinks == [(die_at, [0, 1])]
        assert (w, r) == (2, m)
        assert steps == n_steps
    assert torch.equal(res[0][4], res[1][4])  # survivors hold identical weights
