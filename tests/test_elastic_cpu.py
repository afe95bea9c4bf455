"""Elastic data parallelism (parallel/elastic.py) on gloo: 3 ranks train the Cellpose CPnet; one
member dies mid-run (os._exit right before its step's all-reduce); the survivors detect the failed
collective, agree on the survivor set through the control store, re-init a 2-rank process group,
re-bind the trainer (bucketed all-reduce + weight/moment broadcast) and finish every step with
identical weights.  The control store lives in this (launcher) process, so killing original rank 0
is survivable too."""
import hashlib
import os

import pytest
import torch
import torch.multiprocessing as mp


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
    # plain picklable data only: a torch tensor would travel as a shm fd that dies with this process
    digest = hashlib.sha256(tr.fp.flat.detach().cpu().numpy().tobytes()).hexdigest()
    q.put((member, losses, shrinks, ew.world, ew.rank, digest, tr.step_count))
    ew.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("victim", [2, 0])
def test_elastic_shrink_on_rank_failure(victim):
    from bioengine_worker_amd.parallel.elastic import ControlStore

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = ControlStore()  # hosted by the launcher, not by any training rank
    world, die_at, n_steps = 3, 2, 5
    ps = [ctx.Process(target=_worker, args=(m, world, store.port, q, victim, die_at, n_steps)) for m in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world - 1):
        m, losses, shrinks, w, r, digest, steps = q.get(timeout=240)
        res[m] = (losses, shrinks, w, r, digest, steps)
    for p in ps:
        p.join(60)
    survivors = [m for m in range(world) if m != victim]
    assert ps[victim].exitcode == 17
    assert sorted(res) == survivors
    for m, (losses, shrinks, w, r, digest, steps) in res.items():
        assert len(losses) == n_steps and all(x == x for x in losses)
        assert shrinks == [(die_at, survivors)]
        assert (w, r) == (2, survivors.index(m))
        assert steps == n_steps
    assert res[survivors[0]][4] == res[survivors[1]][4]  # survivors hold identical weights
