"""One rank of a gang job (``serve/gang.py``): ``python -m bioengine_worker_amd.serve.gang_worker``.

Environment (set by the launcher): RANK, WORLD_SIZE, LOCAL_RANK, BE_GANG_STORE=host:port (the
launcher-hosted TCPStore), BE_GANG_BACKEND (nccl | gloo), BE_GANG_DIR (spec.pkl in,
rank<r>.result out).  The process group is initialised before the target runs and destroyed after;
the target is called as ``fn(rank=..., world=..., **kwargs)`` and its return value is pickled back.
"""
from __future__ import annotations

import importlib
import os
import pickle
import sys
import traceback
from datetime import timedelta
from pathlib import Path


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    work = Path(os.environ["BE_GANG_DIR"])
    backend = os.environ.get("BE_GANG_BACKEND", "gloo")
    host, port = os.environ["BE_GANG_STORE"].rsplit(":", 1)
    spec = pickle.loads((work / "spec.pkl").read_bytes())
    out = work / f"rank{rank}.result"
    import torch
    import torch.distributed as dist

    rc = 0
    try:
        if backend == "nccl":
            torch.cuda.set_device(local)
        store = dist.TCPStore(host, int(port), None, False, timedelta(seconds=300))
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, store=dist.PrefixStore("gang", store), rank=rank, world_size=world,
                                timeout=timedelta(seconds=float(os.environ.get("BE_GANG_PG_TIMEOUT_S", "600"))), **kw)
        mod, _, fn_name = spec["target"].partition(":")
        fn = getattr(importlib.import_module(mod), fn_name)
        val = fn(rank=rank, world=world, **spec["kwargs"])
        payload = (True, val)
    except BaseException as e:  # noqa: BLE001
        traceback.print_exc()
        payload = (False, f"{type(e).__name__}: {e}")
        rc = 1
    try:
        data = pickle.dumps(payload)
    except Exception as e:  # noqa: BLE001
        data = pickle.dumps((False, f"result of rank {rank} is not picklable: {e}"))
        rc = 1
    tmp = out.with_suffix(".tmp")
    tmp.write_bytes(data)
    os.replace(tmp, out)
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            if rc == 0:
                dist.barrier()
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass
    sys.stdout.flush()
    return rc


if __name__ == "__main__":
    sys.exit(main())
