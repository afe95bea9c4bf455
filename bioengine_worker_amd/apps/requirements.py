"""Application pip requirements: pinning, resolution against the installed environment, offline
installation from a local wheelhouse, and a clear failure when something cannot be satisfied.

Reference behaviour (``bioengine/utils/requirements.py:10-124``, ``bioengine/apps/builder.py:300-517``):
every deployment's ``ray_actor_options.runtime_env.pip`` list gets the worker's own RPC/serialisation
requirements added (``httpx``, ``hypha-rpc``, ``pydantic``) with ``>=``/``<=``/``~=`` collapsed to
``==`` so replicas resolve to the worker's versions, and Ray installs the list into a per-job
virtualenv.  Here replicas run on the worker's own interpreter, so:

* each requirement is checked against the installed distributions (``importlib.metadata`` +
  ``packaging`` specifiers); the framework's own shims (``ray``, ``hypha-rpc``, ``bioengine``) are
  provided by :mod:`bioengine_worker_amd.compat` and always count as satisfied;
* what is missing is installed from the local wheelhouse(s) in ``BIOENGINE_WHEELHOUSE`` (no index,
  no network) into the application's own ``--target`` directory, which is put on the replicas'
  ``PYTHONPATH`` (and the worker's ``sys.path`` for in-process replicas);
* if anything is still unsatisfied -- no wheelhouse, no matching wheel, or a wheel whose own
  dependencies are missing -- :class:`MissingRequirementsError` lists every missing package and the
  application goes to ``DEPLOY_FAILED`` with that message instead of failing later with an opaque
  ``ImportError`` inside a replica.
"""
from __future__ import annotations

import importlib.metadata as md
import logging
import os
import re
import subprocess
import sys
from pathlib import Path

from packaging.requirements import InvalidRequirement, Requirement
from packaging.utils import canonicalize_name

log = logging.getLogger("bioengine.requirements")

_SPLIT = re.compile(r"(==|>=|<=|~=|>|<)")
#: provided by the framework itself (compat shims / this package), never installed
PROVIDED = {"ray", "ray-serve", "hypha-rpc", "bioengine", "bioengine-worker", "bioengine-worker-amd"}
#: what every deployment needs from the worker's environment (reference select list)
WORKER_REQUIREMENTS = ("httpx", "hypha-rpc", "pydantic")


class MissingRequirementsError(RuntimeError):
    def __init__(self, missing: list[tuple[str, str]], detail: str = ""):
        self.missing = missing
        lines = "; ".join(f"{r} ({why})" for r, why in missing)
        super().__init__(f"Missing pip requirements: {lines}" + (f". {detail}" if detail else ""))


def normalize_requirement(requirement: str) -> str:
    """``>=``, ``<=`` and ``~=`` pinned to ``==`` (the lower/upper bound itself)."""
    if not requirement:
        return requirement
    return requirement.replace(">=", "==").replace("<=", "==").replace("~=", "==")


def _name(req: str) -> str:
    return canonicalize_name(_SPLIT.split(req.split(";")[0].split("[")[0].strip(), maxsplit=1)[0].strip())


def get_pip_requirements(select: list[str] | None = None) -> list[str]:
    """The worker's versions of ``select`` (default :data:`WORKER_REQUIREMENTS`) as ``name==version``;
    packages provided by the framework are skipped."""
    out = []
    for n in select or WORKER_REQUIREMENTS:
        if canonicalize_name(n) in PROVIDED:
            continue
        try:
            out.append(f"{n}=={md.version(n)}")
        except md.PackageNotFoundError:
            continue
    return out


def update_requirements(requirements: list[str], select: list[str] | None = None) -> list[str]:
    """Add the worker's pinned requirements that ``requirements`` does not already name."""
    have = {_name(r) for r in requirements if r}
    out = list(requirements)
    for r in get_pip_requirements(select):
        if _name(r) not in have:
            out.append(normalize_requirement(r))
    return out


#: app site-packages directories this process put on sys.path: one app's installs never satisfy
#: another app's requirements (its process replicas would not see them)
_APP_PATHS: set[str] = set()


def _installed_version(name: str, paths: list[str] | None = None) -> str | None:
    search = list(paths or []) + [p for p in sys.path if p not in _APP_PATHS]
    for d in md.distributions(path=search):
        if canonicalize_name(d.metadata["Name"] or "") == name:
            return d.version
    return None


def resolve(requirements: list[str], extra_paths: list[str] | None = None) -> tuple[list[str], list[tuple[str, str]]]:
    """Split ``requirements`` into (satisfied, missing[(requirement, reason)]) against the installed
    distributions plus any ``extra_paths`` (an application's target directory)."""
    ok, missing = [], []
    for raw in requirements:
        raw = (raw or "").strip()
        if not raw or raw.startswith("#"):
            continue
        try:
            req = Requirement(raw)
        except InvalidRequirement as e:
            missing.append((raw, f"invalid requirement: {e}"))
            continue
        if req.marker is not None and not req.marker.evaluate():
            ok.append(raw)  # not for this platform / interpreter
            continue
        name = canonicalize_name(req.name)
        if name in PROVIDED:
            ok.append(raw)
            continue
        ver = _installed_version(name, extra_paths)
        if ver is None:
            missing.append((raw, "not installed"))
        elif req.specifier and not req.specifier.contains(ver, prereleases=True):
            missing.append((raw, f"installed {ver} does not satisfy {req.specifier}"))
        else:
            ok.append(raw)
    return ok, missing


def shadowed(requirements: list[str]) -> list[tuple[str, str]]:
    """Requirements whose distribution the WORKER environment already has at a version that does not
    satisfy them.  An in-process replica would import the worker's copy whatever the app's target
    directory holds (``import`` finds site-packages first), so such an app must run as a process
    replica with its target at the front of PYTHONPATH."""
    out = []
    for raw in requirements or []:
        raw = (raw or "").strip()
        if not raw or raw.startswith("#"):
            continue
        try:
            req = Requirement(raw)
        except InvalidRequirement:
            continue
        if req.marker is not None and not req.marker.evaluate():
            continue
        name = canonicalize_name(req.name)
        if name in PROVIDED or not req.specifier:
            continue
        ver = _installed_version(name, None)
        if ver is not None and not req.specifier.contains(ver, prereleases=True):
            out.append((raw, f"worker has {ver}"))
    return out


def invalid_requirements(requirements: list[str]) -> list[tuple[str, str]]:
    """Entries that must never reach the pip command line: unparsable strings (pip would read
    ``--target=/x``, ``-e path`` or ``--find-links=...`` as options) and direct-URL requirements
    (``pkg @ https://...`` / ``file:///...sdist`` bypass ``--no-index`` and may run build code)."""
    bad = []
    for raw in requirements:
        raw = (raw or "").strip()
        if not raw or raw.startswith("#"):
            continue
        if raw.startswith("-"):
            bad.append((raw, "pip options are not accepted as requirements"))
            continue
        try:
            req = Requirement(raw)
        except InvalidRequirement as e:
            bad.append((raw, f"invalid requirement: {e}"))
            continue
        if req.url:
            bad.append((raw, "direct-URL requirements are not installable offline from the wheelhouse"))
    return bad


def wheelhouses() -> list[str]:
    v = os.environ.get("BIOENGINE_WHEELHOUSE", "")
    return [p for p in v.split(os.pathsep) if p and Path(p).is_dir()]


def _requires_of_target(target: Path) -> list[str]:
    """Runtime dependencies declared by the distributions installed into ``target``."""
    out = []
    for d in md.distributions(path=[str(target)]):
        for r in d.requires or []:
            try:
                req = Requirement(r)
            except InvalidRequirement:
                continue
            if req.marker is not None and not req.marker.evaluate({"extra": ""}):
                continue
            out.append(str(req).split(";")[0].strip())
    return out


def env_target(requirements: list[str]) -> Path:
    """Shared install directory of one ``runtime_env.pip`` set (keyed by the pinned requirements),
    under ``BIOENGINE_ENV_CACHE`` (default ``~/.bioengine/envs``)."""
    import hashlib

    key = hashlib.sha1("\n".join(sorted(update_requirements(list(requirements)))).encode()).hexdigest()[:16]
    root = Path(os.environ.get("BIOENGINE_ENV_CACHE", Path.home() / ".bioengine" / "envs"))
    return root / key


def runtime_env_path(runtime_env: dict | None) -> str | None:
    """Satisfy a task's ``runtime_env["pip"]`` (reference: Ray installs it per task/actor) and return
    the directory a child process must put on PYTHONPATH (None when nothing had to be installed).
    Raises :class:`MissingRequirementsError` naming what stays unsatisfied."""
    reqs = list((runtime_env or {}).get("pip") or [])
    if isinstance((runtime_env or {}).get("pip"), dict):  # {"packages": [...]} form
        reqs = list(runtime_env["pip"].get("packages") or [])
    if not reqs:
        return None
    info = ensure(reqs, env_target(reqs), add_to_sys_path=False)
    return info["target"]


def ensure(requirements: list[str], target: str | Path, wheel_dirs: list[str] | None = None,
           timeout_s: float = 600.0, add_to_sys_path: bool = True) -> dict:
    """Satisfy ``requirements`` for one application (blocking; run it in a thread).

    Returns ``{"pinned", "satisfied", "installed", "target"}``; raises
    :class:`MissingRequirementsError` listing everything that stays unsatisfied."""
    target = Path(target)
    pinned = update_requirements(list(requirements or []))
    bad = invalid_requirements(pinned)
    if bad:  # never hand these to pip: "--target=..." / "-e path" would be read as options
        raise MissingRequirementsError(bad, "rejected before install")
    paths = [str(target)] if target.is_dir() else []
    _, missing = resolve(pinned, paths)
    installed: list[str] = []
    wheel_dirs = wheelhouses() if wheel_dirs is None else [w for w in wheel_dirs if Path(w).is_dir()]
    if missing and wheel_dirs:
        target.mkdir(parents=True, exist_ok=True)
        reqs = [str(Requirement(r)) for r, _ in missing]
        # dependencies of the wheels are resolved against the worker environment + target below,
        # so pip installs only what was asked for (an index-free resolver cannot see site-packages
        # from a --target install)
        cmd = [sys.executable, "-m", "pip", "install", "--no-index", "--no-deps", "--disable-pip-version-check",
               "--no-cache-dir", "--target", str(target), "--upgrade"]
        for w in wheel_dirs:
            cmd += ["--find-links", w]
        cmd += ["--"] + reqs
        log.info("installing %s from %s into %s", reqs, wheel_dirs, target)
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
        if p.returncode != 0:
            tail = (p.stderr or p.stdout).strip().splitlines()[-3:]
            _, still = resolve(pinned, [str(target)])
            raise MissingRequirementsError(still or missing, "wheelhouse install failed: " + " | ".join(tail))
        installed = reqs
        paths = [str(target)]
        _, missing = resolve(pinned, paths)
        # the installed wheels' own runtime dependencies must be importable too
        if not missing:
            _, dep_missing = resolve(_requires_of_target(target), paths)
            missing = [(r, f"dependency of an installed wheel: {why}") for r, why in dep_missing]
    if missing:
        detail = ("no wheelhouse configured (set BIOENGINE_WHEELHOUSE to a directory of wheels)"
                  if not wheel_dirs else f"not satisfiable from the wheelhouse {wheel_dirs}")
        raise MissingRequirementsError(missing, detail)
    shadow = shadowed(pinned)
    if shadow:
        log.warning("requirements %s conflict with the worker's own packages: the app runs as a process "
                    "replica (target first on PYTHONPATH), never in-process", shadow)
    if paths and add_to_sys_path and not shadow:  # in-process replicas import from the target too
        # appended, not prepended: a package an app installs must never replace a module the worker
        # (or another in-process app) already imports; process replicas get the target at the FRONT
        # of their own PYTHONPATH instead (serve/replica.py), where it affects nobody else
        _APP_PATHS.add(paths[0])
        if paths[0] not in sys.path:
            sys.path.append(paths[0])
    return {"pinned": pinned, "satisfied": True, "installed": installed, "target": paths[0] if paths else None,
            "shadowed": [r for r, _ in shadow]}
