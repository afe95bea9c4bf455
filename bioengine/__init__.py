"""`bioengine` import surface used by app code written for the reference
(``from bioengine import __version__``, ``from bioengine.utils import create_logger``, ...).
Everything is implemented in :mod:`bioengine_worker_amd`; this package only re-exports it."""
from bioengine_worker_amd import __version__  # noqa: F401
