"""Elastic data parallelism: survive a rank failure by shrinking the world to the survivors.

The reference has no multi-GPU training at all (SURVEY.md §2.7, §5 "Failure detection": "RCCL
communicator abort + re-init on rank failure (elastic shrink to N-1 GPUs for DP)" is a new-build
item).  Design, one process per GPU as everywhere else:

* **Control store.**  A ``TCPStore`` hosted OUTSIDE the training ranks -- by the launcher (the
  gang launcher in ``serve/gang.py`` or a test parent, via :class:`ControlStore`) -- so any rank,
  original rank 0 included, can die without taking the store with it.  Every generation of the
  process group rendezvouses under its own ``PrefixStore("pg<gen>")`` so a re-init never sees
  stale keys.  (``host_store=True`` keeps the old single-host mode for ad-hoc runs.)
* **Heartbeats.**  Each rank increments a counter ``hb/<id>`` every ``heartbeat_s`` from a daemon
  thread.  Observers never compare clocks across hosts: each remembers, on its OWN monotonic
  clock, when it last saw a member's counter change, and a member is stale when its counter has
  not moved for ``stale_s``.  When a current member goes stale while a collective may be blocked
  on it, the communicator is *aborted* (RCCL ``abort`` through ``_abort_process_group``) so the
  blocked ``wait()`` raises instead of hanging for the PG timeout.  Gloo fails fast on its own.
* **Agreement.**  Survivors announce themselves under ``gen<g+1>/alive/<id>``, wait until every
  member either announced or has a stale heartbeat, and the first survivor to finish publishes its
  view with ``compare_set(gen<g+1>/members)`` — every survivor adopts that single decision
  (a rank announced too late finds itself excluded and stops).
* **Re-init.**  Survivors re-rank contiguously in original-id order, ``init_process_group`` with
  the new world size, and the trainer re-binds its bucketed all-reduce and broadcasts weights,
  AdamW moments and BN buffers from the new rank 0 (survivors are identical anyway: a step that
  failed mid-all-reduce never reached the optimizer).  The per-rank batch stays fixed, so the
  global batch shrinks with the world (the step's gradient is still a mean over ranks).

Identity: ``member_id`` is the original rank and never changes; ``rank``/``world`` are the current
generation's.  Works on gloo (CPU tests) and nccl (= RCCL).
"""
from __future__ import annotations

import json
import os
import threading
import time
from datetime import timedelta

import torch
import torch.distributed as dist


class ExcludedFromWorld(RuntimeError):
    """This rank was declared dead by the survivors (e.g. it stalled past the heartbeat window)."""


class ControlStore:
    """The elastic control store, hosted by a process that is not a training rank (the launcher).
    Keep the object alive for the lifetime of the job; ``port`` is what ranks connect to."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, timeout_s: float = 120.0):
        self.store = dist.TCPStore(host, port, None, True, timedelta(seconds=timeout_s), wait_for_workers=False)
        self.host, self.port = host, self.store.port


class ElasticWorld:
    def __init__(self, member_id: int, world_size: int, master_addr: str = "127.0.0.1", master_port: int = 29600,
                 backend: str | None = None, heartbeat_s: float = 0.5, stale_s: float = 3.0,
                 pg_timeout_s: float = 30.0, device: torch.device | None = None, host_store: bool = False):
        self.member_id = int(member_id)
        self.members = list(range(int(world_size)))
        self.backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        self.heartbeat_s, self.stale_s, self.pg_timeout_s = heartbeat_s, stale_s, pg_timeout_s
        self.device = device
        self.gen = 0
        self.store = dist.TCPStore(master_addr, master_port, None, bool(host_store),
                                   timedelta(seconds=max(60.0, pg_timeout_s)), wait_for_workers=False)
        self._seen: dict[int, tuple[int, float]] = {}  # member -> (last counter, local monotonic time it moved)
        self._seen_lock = threading.Lock()
        self._stop = threading.Event()
        self._beat()
        self._hb = threading.Thread(target=self._heartbeat_loop, daemon=True)
        self._hb.start()
        self.aborts = 0
        self._init_pg()

    # ------------------------------------------------------------------ membership
    @property
    def rank(self) -> int:
        return self.members.index(self.member_id)

    @property
    def world(self) -> int:
        return len(self.members)

    def _init_pg(self) -> None:
        kw = {}
        if self.backend == "nccl" and self.device is not None:
            kw["device_id"] = self.device
        dist.init_process_group(self.backend, store=dist.PrefixStore(f"pg{self.gen}", self.store), rank=self.rank,
                                world_size=self.world, timeout=timedelta(seconds=self.pg_timeout_s), **kw)

    def _beat(self) -> None:
        self.store.add(f"hb/{self.member_id}", 1)

    def _counter(self, m: int) -> int:
        try:
            return self.store.add(f"hb/{m}", 0)
        except Exception:  # noqa: BLE001
            return -1

    def stale_members(self) -> list[int]:
        """Members whose heartbeat counter has not moved for ``stale_s`` on THIS process's
        monotonic clock (no cross-host wall-clock comparison)."""
        now = time.monotonic()
        out = []
        with self._seen_lock:
            for m in self.members:
                if m == self.member_id:
                    continue
                c = self._counter(m)
                last = self._seen.get(m)
                if last is None or c != last[0]:
                    self._seen[m] = (c, now)
                elif now - last[1] > self.stale_s:
                    out.append(m)
        return out

    def _heartbeat_loop(self) -> None:
        while not self._stop.wait(self.heartbeat_s):
            try:
                self._beat()
                stale = self.stale_members()
                if self.backend == "nccl" and dist.is_initialized() and stale:
                    self._abort()  # unblock a collective waiting on a dead peer
            except Exception:  # noqa: BLE001  (store gone: the launcher died; nothing to do)
                pass

    def _abort(self) -> None:
        self.aborts += 1
        try:
            from torch.distributed.distributed_c10d import _abort_process_group

            _abort_process_group()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------ recovery
    def shrink(self, join_timeout_s: float | None = None) -> list[int]:
        """Tear down the broken group, agree on the survivors, re-init.  Returns the new members."""
        g = self.gen + 1
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
        self.store.set(f"gen{g}/alive/{self.member_id}", "1")
        deadline = time.time() + (join_timeout_s or 4 * self.stale_s + 10)
        decided = None
        while decided is None:
            if self.store.check([f"gen{g}/members"]):
                decided = json.loads(self.store.get(f"gen{g}/members").decode())
                break
            alive = [m for m in self.members if self.store.check([f"gen{g}/alive/{m}"])]
            stale = set(self.stale_members())
            if all(m in alive or m in stale for m in self.members) or time.time() > deadline:
                mine = json.dumps(sorted(alive))
                got = self.store.compare_set(f"gen{g}/members", "", mine)
                decided = json.loads(got.decode() if isinstance(got, bytes) else got)
                break
            time.sleep(0.05)
        if self.member_id not in decided:
            self.close()
            raise ExcludedFromWorld(f"member {self.member_id} excluded at generation {g}: {decided}")
        self.members, self.gen = list(decided), g
        self._init_pg()
        return self.members

    def close(self) -> None:
        self._stop.set()
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def run_elastic(world: ElasticWorld, trainer, batches, n_steps: int, on_shrink=None) -> list[float]:
    """Train ``n_steps`` with ``trainer.step(*batches(step, world))``; on a collective failure
    shrink the world, re-bind the trainer and retry the same step.  Returns the per-step losses."""
    losses: list[float] = []
    step = 0
    while step < n_steps:
        try:
            loss = trainer.step(*batches(step, world))
            losses.append(float(loss))
            step += 1
        except ExcludedFromWorld:
            raise
        except Exception as e:  # noqa: BLE001  (peer died mid-collective: RuntimeError / DistBackendError)
            members = world.shrink()
            trainer.rebind(world.world, world.rank, None)
            if on_shrink is not None:
                on_shrink(step, members, e)
    return losses
