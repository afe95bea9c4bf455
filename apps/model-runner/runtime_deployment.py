"""GPU runtime of the model runner (reference apps/model-runner/runtime_deployment.py:31-312).

``predict`` builds (and caches, ``@serve.multiplexed`` LRU of ``PIPELINE_CACHE_SIZE`` = 10
pipelines as in the reference) a :class:`PredictionPipeline` per (package, weights format,
device, blocksize, package modification time) and runs the sample; ``test`` runs
:func:`test_model`.  Out-of-memory errors are re-raised as plain ``RuntimeError`` so they cross the
RPC boundary cleanly (reference :296-312).
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
from typing import Dict, List, Optional, Union

import numpy as np
from ray import serve

logger = logging.getLogger("ray.serve")


@serve.deployment(
    ray_actor_options={"num_cpus": 1, "num_gpus": 1, "memory": 12 * 1024 ** 3},
    max_ongoing_requests=1,
    autoscaling_config={"min_replicas": 1, "initial_replicas": 1, "max_replicas": 2,
                        "target_num_ongoing_requests_per_replica": 0.8},
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

    async def test(self, rdf_path: str, additional_requirements: Optional[List[str]] = None) -> dict:
        from bioengine_worker_amd.bioimageio.testing import test_model

        if additional_requirements:
            logger.info("additional requirements are not installed by this runtime (offline): %s", additional_requirements)
        return test_model(os.path.dirname(rdf_path) if rdf_path.endswith(".yaml") else rdf_path)

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
        return PredictionPipeline(os.path.dirname(src) if src.endswith(".yaml") else src,
                                  device=kw["device"], weights_format=kw["weights_format"],
                                  default_blocksize_parameter=kw["default_blocksize_parameter"])

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
            return pipe.predict(inputs)
        except Exception as e:  # noqa: BLE001
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
            if "out of memory" in str(e).lower() or type(e).__name__ in ("OutOfMemoryError",):
                raise RuntimeError(f"GPU out of memory during inference: {e}") from None
            raise
