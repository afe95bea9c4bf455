"""Datasets: client (``BioEngineDatasets``), HTTP zarr store + chunk cache, FastAPI server."""
from .client import BioEngineDatasets  # noqa: F401
from .store import ChunkCache, HttpZarrStore, read_zarr_array, write_zarr_array  # noqa: F401
