from bioengine_worker_amd.worker.worker import BioEngineWorker  # noqa: F401
