from bioengine_worker_amd.apps.builder import AppBuilder  # noqa: F401
from bioengine_worker_amd.apps.manager import AppsManager  # noqa: F401
