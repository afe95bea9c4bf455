"""Hypha-compatible transport: in-process hub, WebSocket hub server/client, schema decorators."""
from .client import ServiceProxy, connect_to_server  # noqa: F401
from .hub import Hub, ObjDict, get_local_hub  # noqa: F401
from .schema import schema_function, schema_method  # noqa: F401
