"""``schema_method`` / ``schema_function`` — JSON-schema annotated service methods.

App code written for the reference imports ``from hypha_rpc.utils.schema import schema_method`` and
declares parameters with ``pydantic.Field`` defaults (e.g. ``apps/demo-app/demo_deployment.py``);
the builder collects each entry method's ``__schema__`` to publish the app service interface
(``bioengine/apps/builder.py:1453-1465``).  This module provides the same decorator semantics:

* ``__schema__``: ``{"name", "description", "parameters": {"type": "object", "properties", "required"}}``
  built from the signature, type hints, ``Field(description=..., default=...)`` and the docstring;
* calls substitute ``Field`` defaults with their real default values, so the function body never
  sees a ``FieldInfo``;
* ``context`` parameters are hidden from the schema (they are injected by the RPC layer).
"""
from __future__ import annotations

import functools
import inspect
import typing
from typing import Any

try:
    from pydantic.fields import FieldInfo
    from pydantic_core import PydanticUndefined
except Exception:  # pragma: no cover
    FieldInfo = ()  # type: ignore
    PydanticUndefined = object()  # type: ignore

_HIDDEN = {"self", "cls", "context"}


def _json_type(tp) -> dict:
    origin = typing.get_origin(tp)
    args = typing.get_args(tp)
    if tp in (inspect.Parameter.empty, Any, None):
        return {}
    if origin is typing.Union:
        non_none = [a for a in args if a is not type(None)]
        if len(non_none) == 1:
            return _json_type(non_none[0])
        return {"anyOf": [_json_type(a) for a in non_none]}
    if tp is str:
        return {"type": "string"}
    if tp is bool:
        return {"type": "boolean"}
    if tp is int:
        return {"type": "integer"}
    if tp is float:
        return {"type": "number"}
    if tp in (list, tuple) or origin in (list, tuple):
        d = {"type": "array"}
        if args:
            d["items"] = _json_type(args[0])
        return d
    if tp is dict or origin is dict:
        return {"type": "object"}
    if origin is typing.Literal:
        return {"enum": list(args)}
    return {}


def _field_default(v):
    if isinstance(v, FieldInfo):
        d = v.default
        if d is PydanticUndefined:
            if v.default_factory is not None:
                return v.default_factory()
            return inspect.Parameter.empty
        return d
    return v


def build_schema(fn) -> dict:
    sig = inspect.signature(fn)
    try:
        hints = typing.get_type_hints(fn)
    except Exception:
        hints = {}
    props, required = {}, []
    for name, p in sig.parameters.items():
        if name in _HIDDEN or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
            continue
        prop = _json_type(hints.get(name, p.annotation))
        default = p.default
        if isinstance(default, FieldInfo):
            if default.description:
                prop["description"] = default.description
            d = _field_default(default)
            if d is inspect.Parameter.empty:
                required.append(name)
            else:
                prop["default"] = d
        elif default is inspect.Parameter.empty:
            required.append(name)
        else:
            try:
                import json

                json.dumps(default)
                prop["default"] = default
            except TypeError:
                pass
        props[name] = prop
    doc = inspect.getdoc(fn) or ""
    return {"name": fn.__name__, "description": doc.strip(),
            "parameters": {"type": "object", "properties": props, "required": required}}


def _bind_defaults(fn, sig, args, kwargs):
    bound = sig.bind_partial(*args, **kwargs)
    for name, p in sig.parameters.items():
        if name not in bound.arguments and isinstance(p.default, FieldInfo):
            d = _field_default(p.default)
            if d is inspect.Parameter.empty:
                if name == "context":
                    bound.arguments[name] = None
                    continue
                raise TypeError(f"{fn.__name__}() missing required argument: '{name}'")
            bound.arguments[name] = d
    return bound.args, bound.kwargs


def _defaults_binder(fn, sig):
    """Per-call Field-default filling without ``Signature.bind`` (which costs ~20-80 us per request
    on the serving hot path): positions and defaults are resolved once at decoration time; a call
    with unknown keywords or a signature with *args/**kwargs takes the general path."""
    params = list(sig.parameters.values())
    if any(p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD, p.POSITIONAL_ONLY) for p in params):
        return lambda args, kwargs: _bind_defaults(fn, sig, args, kwargs)
    names = {p.name for p in params}
    fields = []
    for i, p in enumerate(params):
        if isinstance(p.default, FieldInfo):
            fi = p.default
            const = fi.default is not PydanticUndefined or fi.default_factory is None
            fields.append((i, p.name, fi, const, fi.default if fi.default is not PydanticUndefined else inspect.Parameter.empty))

    def bind(args, kwargs):
        if any(k not in names for k in kwargs):
            return _bind_defaults(fn, sig, args, kwargs)
        n = len(args)
        out = None
        for i, name, fi, const, d in fields:
            if i < n or name in kwargs:
                continue
            v = d if const else fi.default_factory()
            if v is inspect.Parameter.empty:
                if name != "context":
                    raise TypeError(f"{fn.__name__}() missing required argument: '{name}'")
                v = None
            if out is None:
                out = dict(kwargs)
            out[name] = v
        return args, (kwargs if out is None else out)

    return bind


def schema_method(fn=None, **_opts):
    """Decorator for (async) methods/functions; attaches ``__schema__`` and resolves Field defaults."""
    if fn is None:
        return lambda f: schema_method(f, **_opts)
    sig = inspect.signature(fn)
    bind = _defaults_binder(fn, sig)
    if inspect.iscoroutinefunction(fn):
        @functools.wraps(fn)
        async def wrapper(*args, **kwargs):
            a, k = bind(args, kwargs)
            return await fn(*a, **k)
    else:
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            a, k = bind(args, kwargs)
            return fn(*a, **k)
    wrapper.__schema__ = build_schema(fn)
    wrapper.__is_schema_method__ = True
    return wrapper


schema_function = schema_method
