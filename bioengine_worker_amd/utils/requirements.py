"""Pip requirement pinning for app runtime environments (reference: bioengine/utils/requirements.py).

``get_pip_requirements`` pins the worker's own dependencies (selected by name) to the versions
installed here, so app replicas import the same client libraries.  ``update_requirements`` merges
two requirement lists without overriding entries already present in the first.
"""
from __future__ import annotations

import re
from importlib import metadata

_NAME = re.compile(r"^\s*([A-Za-z0-9_.\-]+)")


def _name(req: str) -> str:
    m = _NAME.match(req)
    return (m.group(1) if m else req).lower().replace("_", "-")


def get_pip_requirements(select: list[str] | None = None, exclude: tuple[str, ...] = ("ray",)) -> list[str]:
    out = []
    for name in select or []:
        n = _name(name)
        if n in exclude:
            continue
        try:
            out.append(f"{n}=={metadata.version(n)}")
        except metadata.PackageNotFoundError:
            continue
    return out


def update_requirements(base: list[str] | None, extra: list[str] | None) -> list[str]:
    base = list(base or [])
    have = {_name(r) for r in base}
    for r in extra or []:
        if _name(r) not in have:
            base.append(r)
            have.add(_name(r))
    return base
