"""Data-parallel fine-tuning correctness on gloo (CPU):

* a stop requested at a random step ends every rank of a 3-rank gang within seconds (the stop flag is
  decided collectively with the loss all-reduce, so no rank is left waiting in a collective);
* Cellpose-SAM (tiny) at world 2 ends with the same weights as world 1 on the doubled batch;
* killing one of 3 ranks restarts a fresh gang at world 2 from the last epoch checkpoint, and the
  session completes (elastic restart, ``train/session.py:run_dp_session``).
"""
import asyncio
import json
import os
import random
import time
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _session(tmp_path: Path, n=6, size=64, model="cyto3", n_epochs=3, **extra) -> tuple[Path, dict]:
    from bioengine_worker_amd.train.cellpose_train import synthetic_instances

    sdir = tmp_path / "sessions" / "s1"
    (sdir / "data").mkdir(parents=True)
    ims, labs = synthetic_instances(n, size, size, ncells=8, seed=1)
    pairs = []
    for i in range(n):
        ip, lp = sdir / "data" / f"im{i}.npy", sdir / "data" / f"lab{i}.npy"
        np.save(ip, (ims[i, 0] * 1000 + 200).astype(np.float32))
        np.save(lp, labs[i].astype(np.int32))
        pairs.append({"image": str(ip), "annotation": str(lp)})
    (sdir / "pairs.json").write_text(json.dumps({"train": pairs, "test": []}))
    params = {"model": model, "n_epochs": n_epochs, "batch_size": 1, "learning_rate": 1e-4, "weight_decay": 1e-4,
              "min_train_masks": 1, "bsize": 32, **extra}
    (sdir / "status.json").write_text(json.dumps({"status_type": "preparing"}))
    return sdir, params


def _fresh_gang_manager():
    from bioengine_worker_amd.serve import gang
    from bioengine_worker_amd.serve.controller import ResourcePool

    gang._local = gang.GangManager(ResourcePool(gpu_ids=[]))
    return gang._local


@pytest.mark.timeout(600)
def test_stop_at_random_step_ends_all_ranks(tmp_path):
    from bioengine_worker_amd.train.session import read_status, run_dp_session

    _fresh_gang_manager()
    sdir, params = _session(tmp_path, n=9, n_epochs=200)

    async def main():
        task = asyncio.ensure_future(run_dp_session(sdir, params, 3, max_restarts=0, gpus_per_rank=0))
        # wait until training steps are running, then stop at a random moment
        t0 = time.time()
        while time.time() - t0 < 240:
            st = read_status(sdir)
            if st.get("status_type") == "running" and (st.get("current_batch") or 0) >= 1:
                break
            await asyncio.sleep(0.1)
        await asyncio.sleep(random.uniform(0.2, 1.5))
        (sdir / "stop").touch()
        ts = time.time()
        res = await asyncio.wait_for(task, 120)
        return time.time() - ts, res

    dt, res = asyncio.run(main())
    assert dt < 5.0, f"ranks took {dt:.1f} s to stop"
    assert len(res) == 3 and all(r["status_type"] in (None, "stopped") for r in res[1:])
    assert read_status(sdir)["status_type"] == "stopped"
    # every rank stopped with identical weights (same number of steps taken)
    assert len({r["weights_sha256"] for r in res}) == 1


@pytest.mark.timeout(600)
def test_rank_kill_restarts_at_smaller_world_and_completes(tmp_path):
    from bioengine_worker_amd.train.session import read_status, run_dp_session

    _fresh_gang_manager()
    sdir, params = _session(tmp_path, n=6, n_epochs=3, fault_injection={"kill_rank": 2, "at_batch": 4})
    res = asyncio.run(asyncio.wait_for(run_dp_session(sdir, params, 3, gpus_per_rank=0), 500))
    st = read_status(sdir)
    assert st["status_type"] == "completed", st
    assert st["elastic_restarts"] == 1 and st["world_size"] == 2
    assert len(res) == 2 and res[0]["weights_sha256"] == res[1]["weights_sha256"]
    assert len(st["train_losses"]) == 3 and all(np.isfinite(st["train_losses"]))


# ---------------------------------------------------------------------------- DP == doubled batch
def _tiny_cpsam():
    from bioengine_worker_amd.cellpose.model_store import CPSAM_ARCHS, new_net

    net = new_net("cpsam", dict(CPSAM_ARCHS["tiny"], bsize=32))
    torch.manual_seed(0)
    for p in net.parameters():
        p.data.normal_(0, 0.05) if p.dim() > 1 else p.data.normal_(0, 0.01)
    net.rdrop = 0.0
    return net


def _crops(n, S, seed=7):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, S, S, generator=g)
    lbl = torch.zeros(n, 3, S, S)
    lbl[:, 0] = (torch.rand(n, S, S, generator=g) > 0.6).float()
    lbl[:, 1:] = 0.3 * torch.randn(n, 2, S, S, generator=g)
    return x, lbl


def _cpsam_worker(rank, world, port, q, B, steps, S):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bioengine_worker_amd.train.cellpose_train import CellposeTrainer, TrainConfig

        tr = CellposeTrainer(_tiny_cpsam(), TrainConfig(batch_size=B, bsize=S, lr=1e-3, weight_decay=1e-4,
                                                        bucket_mb=0.05), "cpu", world_size=world, rank=rank)
        losses = []
        for k in range(steps):
            x, lbl = _crops(B * world, S, seed=10 + k)
            loss = tr._step_cpsam(x[rank * B:(rank + 1) * B], lbl[rank * B:(rank + 1) * B])
            losses.append(tr.agree(loss, B)[0])
        q.put((rank, tr.fp.flat.numpy().copy(), losses))
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 -- report instead of leaving the parent waiting
        import traceback

        q.put((rank, None, traceback.format_exc()))
        raise


@pytest.mark.timeout(600)
def test_cpsam_dp_world2_equals_world1_doubled_batch():
    from bioengine_worker_amd.train.cellpose_train import CellposeTrainer, TrainConfig

    B, steps, S, world = 2, 3, 32, 2
    port = 29300 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpsam_worker, args=(r, world, port, q, B, steps, S)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
    for rank, flat, info in res:
        assert flat is not None, info
    tr = CellposeTrainer(_tiny_cpsam(), TrainConfig(batch_size=B * world, bsize=S, lr=1e-3, weight_decay=1e-4),
                         "cpu", world_size=1, rank=0)
    losses = []
    for k in range(steps):
        x, lbl = _crops(B * world, S, seed=10 + k)
        losses.append(float(tr._step_cpsam(x, lbl)))
    ref = tr.fp.flat
    for rank, flat, dl in res:
        torch.testing.assert_close(torch.from_numpy(flat), ref, rtol=1e-4, atol=2e-6)
        np.testing.assert_allclose(dl, losses, rtol=1e-5)  # reported loss = global mean
    assert np.array_equal(res[0][1], res[1][1])
