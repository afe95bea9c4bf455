from bioengine_worker_amd.datasets import BioEngineDatasets, HttpZarrStore  # noqa: F401
