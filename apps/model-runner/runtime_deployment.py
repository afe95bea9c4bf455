"""GPU runtime of the model runner (reference apps/model-runner/runtime_deployment.py:31-312).

``predict`` builds (and caches, ``@serve.multiplexed`` LRU of ``PIPELINE_CACHE_SIZE`` = 10
pipelines as in the reference) a :class:`PredictionPipeline` per (package, weights format,
device, blocksize, package modification time) and runs the sample.  Out-of-memory errors are
re-raised as plain ``RuntimeError`` so they cross the RPC boundary cleanly (reference :296-312).

Where this departs from the reference:

* The reference caps the replica at ONE request (``max_ongoing_requests=1``, :40) and runs each
  prediction inline.  Here requests go through ``@serve.batch``: requests queued while the device
  is busy are run together, and requests for the same pipeline whose inputs pad to the same shape
  share one forward (``PredictionPipeline.predict_many``).  The GPU work runs on a worker thread,
  so the replica's event loop (health checks, new requests, batch forming) never blocks behind a
  long tiled prediction.
* ``test(additional_requirements)`` (reference :101-156 runs the test as a Ray task with
  ``runtime_env.pip``): requirements the runtime already satisfies are dropped; the rest are
  installed from the local wheelhouse (``BIOENGINE_WHEELHOUSE``, no index) into a shared per-set
  directory and the test runs in an isolated child process with that directory on its path
  (``serve/tasks.py``, CPU-only like the reference's ``num_gpus=0``).  A requirement that cannot be
  satisfied offline fails the call with the unsatisfied list before anything runs.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os
from typing import Dict, List, Optional, Union

import numpy as np
from ray import serve

logger = logging.getLogger("ray.serve")

#: requests one replica accepts at once (queued ones are batched; the reference allows 1)
MAX_ONGOING = int(os.environ.get("MODEL_RUNNER_MAX_ONGOING", 16))


def _test_in_env(rdf_path: str, device: str = "cpu") -> dict:
    """Body of the isolated test task (module level so the child imports it by reference)."""
    from bioengine_worker_amd.bioimageio.testing import test_model

    return test_model(os.path.dirname(rdf_path) if rdf_path.endswith(".yaml") else rdf_path, device=device)


@serve.deployment(
    ray_actor_options={"num_cpus": 1, "num_gpus": 1, "memory": 12 * 1024 ** 3},
    max_ongoing_requests=MAX_ONGOING,
    autoscaling_config={"min_replicas": 1, "initial_replicas": 1, "max_replicas": 2,
                        "target_num_ongoing_requests_per_replica": 0.8 * MAX_ONGOING},
    health_check_period_s=30.0,
    health_check_timeout_s=30.0,
    graceful_shutdown_timeout_s=120.0,
)
class RuntimeDeployment:
    """Internal deployment running bioimage.io model inference on the framework's kernels."""

    def __init__(self) -> None:
        self._kwargs_cache: dict = {}

    def _memory(self) -> tuple[int, int]:
        import psutil
        import torch

        gpu = torch.cuda.memory_allocated() if torch.cuda.is_available() else 0
        return psutil.Process().memory_info().rss, gpu

    async def check_health(self) -> None:
        return None

    # ------------------------------------------------------------------ test
    async def test(self, rdf_path: str, additional_requirements: Optional[List[str]] = None) -> dict:
        from bioengine_worker_amd.apps.requirements import invalid_requirements, resolve

        if additional_requirements is not None and not isinstance(additional_requirements, list):
            raise ValueError("additional_requirements must be a list of strings.")
        reqs = [r.strip() for r in additional_requirements or [] if r and r.strip()]
        bad = invalid_requirements(reqs)
        if bad:
            raise ValueError(f"invalid additional requirements: {bad}")
        _, missing = await asyncio.to_thread(resolve, reqs)
        extra = [r for r, _ in missing]
        if not extra:  # everything already importable here: test in this replica, off the loop
            from bioengine_worker_amd.bioimageio.testing import test_model

            src = os.path.dirname(rdf_path) if rdf_path.endswith(".yaml") else rdf_path
            return await asyncio.to_thread(test_model, src)
        import ray

        logger.info("running test of %s in an isolated task with %s", rdf_path, extra)
        task = ray.remote(_test_in_env).options(num_cpus=1, num_gpus=0, runtime_env={"pip": extra})
        report = await task.remote(rdf_path, "cpu")
        report["additional_requirements"] = extra
        return report

    # ------------------------------------------------------------------ predict
    def _key(self, **kw) -> str:
        s = json.dumps(kw, sort_keys=True, default=str)
        k = hashlib.md5(s.encode()).hexdigest()
        self._kwargs_cache[k] = kw
        return k

    @serve.multiplexed(max_num_models_per_replica=int(os.environ.get("PIPELINE_CACHE_SIZE", 10)))
    async def _create_prediction_pipeline(self, cache_key: str):
        from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

        kw = self._kwargs_cache.pop(cache_key)
        src = kw["rdf_path"]
        return await asyncio.to_thread(
            PredictionPipeline, os.path.dirname(src) if src.endswith(".yaml") else src, device=kw["device"],
            weights_format=kw["weights_format"], default_blocksize_parameter=kw["default_blocksize_parameter"])

    @serve.batch(max_batch_size=int(os.environ.get("MODEL_RUNNER_MAX_BATCH", 8)), batch_wait_timeout_s=0.005)
    async def _run(self, pipes: list, inputs: list) -> list:
        """One batch of queued requests: grouped per pipeline, each group one ``predict_many``
        (same-shape requests share a forward).  Runs on a worker thread; errors are per group."""
        groups: dict[int, list[int]] = {}
        for i, p in enumerate(pipes):
            groups.setdefault(id(p), []).append(i)

        def work():
            out: list = [None] * len(pipes)
            for idx in groups.values():
                try:
                    res = pipes[idx[0]].predict_many([inputs[i] for i in idx])
                except Exception as e:  # noqa: BLE001 -- delivered to each request of the group
                    res = [e] * len(idx)
                for i, r in zip(idx, res):
                    out[i] = r
            return out

        return await asyncio.to_thread(work)

    async def predict(self, rdf_path: str, inputs: Union[np.ndarray, Dict[str, np.ndarray]],
                      weights_format: Optional[str] = None, device: Optional[str] = None,
                      default_blocksize_parameter: Optional[int] = None, sample_id: str = "sample",
                      latest_remote_modified: Optional[float] = None) -> Dict[str, np.ndarray]:
        import torch

        if not os.path.exists(rdf_path):
            raise FileNotFoundError(f"RDF not found: {rdf_path}")
        try:
            key = self._key(rdf_path=rdf_path, weights_format=weights_format, device=device,
                            default_blocksize_parameter=default_blocksize_parameter,
                            latest_remote_modified=latest_remote_modified)
            pipe = await self._create_prediction_pipeline(key)
            out = await self._run(pipe, inputs)
            if isinstance(out, BaseException):
                raise out
            return out
        except Exception as e:  # noqa: BLE001
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
            if "out of memory" in str(e).lower() or type(e).__name__ in ("OutOfMemoryError",):
                raise RuntimeError(f"GPU out of memory during inference: {e}") from None
            raise

    def get_batch_stats(self) -> dict | None:
        from bioengine_worker_amd.serve.batching import batch_stats

        return batch_stats(self, "_run")
