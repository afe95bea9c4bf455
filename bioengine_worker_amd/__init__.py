"""bioengine_worker_amd — MI355X-native BioEngine worker.

A from-scratch rebuild of the capabilities of aicell-lab/bioengine-worker for AMD Instinct MI355X
(gfx950): the Hypha-RPC ``bioengine-worker`` service API, app manifest/deployment format and CLI are
kept; the Ray / Ray Serve runtime is replaced by a native per-GPU serving runtime, and the compute
paths (Cellpose U-Net, flow dynamics, tiled 2D/3D conv inference, ViT embedding, fused training
ops) are hand-written CDNA4 HIP kernels.
"""
__version__ = "0.1.0"
