"""Import-surface compatibility for app code written against the reference.

``install()`` makes ``ray`` (when the real Ray is absent) and ``hypha_rpc`` (when the real
hypha-rpc is absent) importable, backed by this framework's native serving runtime and hub client.
The ``bioengine`` package itself (``from bioengine import __version__``,
``from bioengine.utils import create_logger``) is provided by the top-level ``bioengine/`` package.
"""
from __future__ import annotations

import importlib.util
import sys
import types

_done = False


def _has_real(name: str) -> bool:
    mod = sys.modules.get(name)
    if mod is not None:
        return not getattr(mod, "__bioengine_shim__", False)
    try:
        return importlib.util.find_spec(name) is not None
    except (ImportError, ValueError):
        return False


def install(force: bool = False) -> None:
    global _done
    if _done and not force:
        return
    _done = True
    if force or not _has_real("ray"):
        from ..serve.ray_compat import build_modules

        for k, m in build_modules().items():
            m.__bioengine_shim__ = True
            sys.modules[k] = m
    if force or not _has_real("hypha_rpc"):
        from ..transport import schema
        from ..transport.client import connect_to_server

        hr = types.ModuleType("hypha_rpc")
        hr.__path__ = []
        utils = types.ModuleType("hypha_rpc.utils")
        utils.__path__ = []
        sch = types.ModuleType("hypha_rpc.utils.schema")
        sch.schema_method = schema.schema_method
        sch.schema_function = schema.schema_function
        utils.schema = sch
        hr.utils = utils
        hr.connect_to_server = connect_to_server
        hr.__bioengine_shim__ = True

        async def login(config=None, **_):
            import os

            return os.environ.get("HYPHA_TOKEN") or os.environ.get("BIOENGINE_TOKEN")

        hr.login = login
        for k, m in {"hypha_rpc": hr, "hypha_rpc.utils": utils, "hypha_rpc.utils.schema": sch}.items():
            m.__bioengine_shim__ = True
            sys.modules[k] = m
