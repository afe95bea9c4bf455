from bioengine_worker_amd.cli import main  # noqa: F401
