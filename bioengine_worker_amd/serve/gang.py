"""Gang-scheduled multi-process jobs: N ranks, one process (and one GPU) each, one process group.

The reference has no multi-GPU job at all: training is one thread on one GPU, ingestion fans out
independent ``@ray.remote(num_gpus=1)`` tasks (``apps/cell-image-search/ingestion.py:451-531``),
SURVEY.md §2.7.  Data-parallel fine-tuning over RCCL and z-slab sharded EM volumes need all their
ranks at once, so the serving runtime gets a gang primitive:

* ``await run_gang("pkg.module:function", kwargs, world_size=N)`` from anywhere -- an app replica
  process forwards the request to its controller over the replica control channel (the same path
  as nested deployment-handle calls); the controller owns the node's resource pool.
* The controller reserves N GPUs (or CPU-only ranks when ``gpus_per_rank=0``) atomically -- all or
  nothing, FIFO with other demands -- and hosts the job's ``TCPStore`` itself, so the rendezvous
  survives any rank (elastic jobs can re-rendezvous through it, ``parallel/elastic.py``).
* Every rank is a FRESH child Python process (``serve/gang_worker.py``) started before anything
  touches a GPU in it, with ``RANK``/``WORLD_SIZE``/``LOCAL_RANK``, ``HIP_VISIBLE_DEVICES`` = the
  gang's GPUs (torchrun layout: rank r drives local device r, RCCL sees its peers over xGMI) and
  ``BE_GANG_STORE=host:port``.  The worker builds the process group (``nccl`` = RCCL with GPUs,
  else ``gloo``) and calls ``function(rank=, world=, **kwargs)``.
* A rank that fails (non-zero exit, signal, or the job deadline) tears the whole gang down:
  the other ranks are terminated (SIGTERM, then SIGKILL), resources are released and the error
  -- with each failed rank's stderr tail -- is raised to the caller.  A retry is a fresh gang of
  fresh processes, never an exec of a process that has used the GPU.

Results: each rank's return value (picklable) comes back in rank order.
"""
from __future__ import annotations

import asyncio
import logging
import os
import pickle
import signal
import sys
import tempfile
import time
import uuid
from pathlib import Path

log = logging.getLogger("bioengine.serve.gang")


class GangError(RuntimeError):
    pass


class GangManager:
    """Launches and supervises gangs on one node's :class:`~.controller.ResourcePool`."""

    def __init__(self, resources, log_dir: str | None = None):
        self.resources = resources
        self.log_dir = Path(log_dir) if log_dir else None
        self._cv: asyncio.Condition | None = None
        self.jobs: dict[str, dict] = {}

    def _cond(self) -> asyncio.Condition:
        if self._cv is None:
            self._cv = asyncio.Condition()
        return self._cv

    async def _reserve(self, world: int, gpus_per_rank: int, cpus_per_rank: float, wait_s: float):
        res = self.resources
        need_gpu = world * gpus_per_rank
        if need_gpu > res.total_gpu:
            raise GangError(f"gang needs {need_gpu} GPUs but the node has {res.total_gpu:g}")
        cpus = min(world * cpus_per_rank, res.total_cpu)
        cv = self._cond()
        t0 = time.time()
        async with cv:
            while not res.can_fit(cpus, need_gpu, 0):
                if time.time() - t0 > wait_s:
                    raise GangError(f"no {need_gpu} free GPUs / {cpus:g} CPUs within {wait_s:.0f} s")
                try:
                    await asyncio.wait_for(cv.wait(), 1.0)
                except asyncio.TimeoutError:
                    pass
            return cpus, need_gpu, res.reserve(cpus, need_gpu, 0)

    async def _release(self, cpus, gpus, ids):
        cv = self._cond()
        async with cv:
            self.resources.release(cpus, gpus, 0, ids)
            cv.notify_all()

    async def run(self, target: str, kwargs: dict | None = None, world_size: int = 1, gpus_per_rank: int = 1,
                  cpus_per_rank: float = 1.0, backend: str | None = None, timeout_s: float | None = None,
                  env: dict | None = None, wait_for_resources_s: float = 3600.0, name: str | None = None) -> list:
        from ..parallel.elastic import ControlStore

        world = int(world_size)
        if world < 1:
            raise ValueError("world_size must be >= 1")
        if gpus_per_rank and self.resources.total_gpu == 0:
            gpus_per_rank = 0  # CPU-only node: gloo ranks
        backend = backend or ("nccl" if gpus_per_rank else "gloo")
        cpus, ngpu, ids = await self._reserve(world, int(gpus_per_rank), cpus_per_rank, wait_for_resources_s)
        job = name or f"gang-{uuid.uuid4().hex[:8]}"
        work = Path(tempfile.mkdtemp(prefix=f"be-{job}-"))
        store = ControlStore("127.0.0.1", 0)
        procs: list[asyncio.subprocess.Process] = []
        info = {"target": target, "world": world, "gpus": list(ids or []), "backend": backend,
                "started": time.time(), "state": "starting"}
        self.jobs[job] = info
        try:
            (work / "spec.pkl").write_bytes(pickle.dumps({"target": target, "kwargs": dict(kwargs or {})}))
            root = str(Path(__file__).resolve().parents[2])
            for r in range(world):
                e = dict(os.environ)
                e.update({k: str(v) for k, v in (env or {}).items()})
                e.update({"RANK": str(r), "WORLD_SIZE": str(world), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(world),
                          "MASTER_ADDR": "127.0.0.1", "BE_GANG_STORE": f"127.0.0.1:{store.port}",
                          "BE_GANG_BACKEND": backend, "BE_GANG_DIR": str(work), "BE_GANG_JOB": job})
                if ids:
                    e["HIP_VISIBLE_DEVICES"] = ",".join(map(str, ids))
                else:
                    e["HIP_VISIBLE_DEVICES"] = ""
                    # CPU ranks share the node's cores: one intra-op pool per rank sized to its share
                    # (N ranks x all-cores pools oversubscribe and every collective waits on the slowest)
                    if "OMP_NUM_THREADS" not in (env or {}):
                        e["OMP_NUM_THREADS"] = str(max(1, int(self.resources.total_cpu // world)))
                e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
                err = open(work / f"rank{r}.err", "wb")
                out = open(work / f"rank{r}.out", "wb")
                p = await asyncio.create_subprocess_exec(sys.executable, "-u", "-m", "bioengine_worker_amd.serve.gang_worker",
                                                         env=e, stdout=out, stderr=err, start_new_session=True)
                err.close()
                out.close()
                procs.append(p)
            info["state"] = "running"
            info["pids"] = [p.pid for p in procs]
            await self._supervise(job, procs, work, timeout_s)
            results = []
            for r in range(world):
                ok, val = pickle.loads((work / f"rank{r}.result").read_bytes())
                if not ok:
                    raise GangError(f"{job} rank {r} failed: {val}")
                results.append(val)
            info["state"] = "completed"
            return results
        except BaseException:
            info["state"] = "failed"
            await self._kill(procs)
            raise
        finally:
            info["ended"] = time.time()
            await self._release(cpus, ngpu, ids)
            self._keep_logs(job, work, world)
            del store

    async def _supervise(self, job, procs, work: Path, timeout_s):
        deadline = time.time() + timeout_s if timeout_s else None
        pending = {asyncio.ensure_future(p.wait()): r for r, p in enumerate(procs)}
        while pending:
            left = None if deadline is None else max(0.0, deadline - time.time())
            done, _ = await asyncio.wait(list(pending), timeout=left, return_when=asyncio.FIRST_COMPLETED)
            if not done:
                raise GangError(f"{job} exceeded its {timeout_s:.0f} s deadline")
            for f in done:
                r = pending.pop(f)
                rc = f.result()
                if rc != 0:
                    tail = (work / f"rank{r}.err").read_bytes()[-3000:].decode(errors="replace")
                    raise GangError(f"{job} rank {r} exited with {rc}; stderr tail:\n{tail}")

    @staticmethod
    async def _kill(procs, grace_s: float = 5.0):
        live = [p for p in procs if p.returncode is None]
        for p in live:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        t0 = time.time()
        while any(p.returncode is None for p in live) and time.time() - t0 < grace_s:
            await asyncio.sleep(0.1)
        for p in live:
            if p.returncode is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                await p.wait()

    def _keep_logs(self, job, work: Path, world: int):
        import shutil

        try:
            if self.log_dir is not None:
                dst = self.log_dir / "gangs" / job
                dst.mkdir(parents=True, exist_ok=True)
                for r in range(world):
                    for ext in ("out", "err"):
                        f = work / f"rank{r}.{ext}"
                        if f.exists():
                            shutil.copy(f, dst / f.name)
            self.jobs[job]["log_tail"] = {
                r: (work / f"rank{r}.err").read_bytes()[-1000:].decode(errors="replace")
                for r in range(world) if (work / f"rank{r}.err").exists()}
        finally:
            shutil.rmtree(work, ignore_errors=True)

    def status(self) -> dict:
        return {k: {kk: vv for kk, vv in v.items() if kk != "log_tail"} for k, v in self.jobs.items()}


_local: GangManager | None = None


def _local_manager() -> GangManager:
    global _local
    if _local is None:
        from .controller import ResourcePool, _detect_gpus

        _local = GangManager(ResourcePool(gpu_ids=_detect_gpus()))
    return _local


async def run_gang(target: str, kwargs: dict | None = None, world_size: int = 1, gpus_per_rank: int = 1,
                   **opts) -> list:
    """Run ``target`` (``"module:function"``) as a gang of ``world_size`` ranks; returns the ranks'
    results.  Inside an app replica the request goes to the controller that owns the GPUs."""
    from . import controller as ctrl

    call = dict(target=target, kwargs=dict(kwargs or {}), world_size=int(world_size), gpus_per_rank=int(gpus_per_rank),
                **opts)
    if ctrl._child_router is not None:
        return await ctrl._child_router.call("__bioengine__", "gang", "run", [], call)
    if ctrl._controller is not None:
        return await ctrl._controller.gangs.run(**call)
    return await _local_manager().run(**call)


def collective_probe(rank: int, world: int, fail_rank: int = -1, payload_mb: float = 1.0) -> dict:
    """Gang self-test target: one all-reduce + all-gather over the job's process group (RCCL on
    GPUs, gloo on CPU); ``fail_rank`` makes that rank raise (tests the teardown path)."""
    import torch
    import torch.distributed as dist

    if rank == fail_rank:
        raise RuntimeError(f"rank {rank} failing on purpose")
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    n = max(1, int(payload_mb * (1 << 20) / 4))
    t = torch.full((n,), float(rank + 1), device=dev)
    t0 = time.perf_counter()
    dist.all_reduce(t)
    got = [torch.zeros(1, device=dev) for _ in range(world)]
    dist.all_gather(got, torch.tensor([float(rank)], device=dev))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return {"rank": rank, "world": world, "sum": float(t[0].item()), "gathered": [float(g.item()) for g in got],
            "backend": dist.get_backend(), "ms": round((time.perf_counter() - t0) * 1e3, 3)}
