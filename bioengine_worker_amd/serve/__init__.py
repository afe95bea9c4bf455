"""Native serving runtime with a Ray-Serve-compatible API (see :mod:`.api`)."""
from .api import (Application, Deployment, batch, delete, deployment, get_app_handle,  # noqa: F401
                  get_multiplexed_model_id, get_replica_context, multiplexed, run, shutdown, status)
from .handle import DeploymentHandle, DeploymentResponse  # noqa: F401
