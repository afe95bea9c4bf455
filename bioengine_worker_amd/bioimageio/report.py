"""Model test reports: environment rows, the local report cache and publishing to the artifact.

Behaviour of the reference's ``EntryDeployment.test`` (apps/model-runner/entry_deployment.py:1151-1182,
1573-1819), re-implemented over this framework's artifact manager (``transport/hub.py``, or Hypha's):

* a report carries ``tested_at`` (epoch seconds of the run) and ``env`` rows ``[package, version,
  build, channel]`` that include the BioImage.IO implementation versions and a ``bioengine`` row;
* the local cache (``.test_cache.json`` next to the package) is reused only while the package's
  remote modification time AND the implementation versions in the cached ``env`` still match;
* publishing writes ``test_report.json`` into the artifact and a compact ``test_summary``
  ``{status, tested_at, env}`` into its manifest, drops the legacy ``test_reports`` / ``test_report``
  / ``score`` manifest keys and the legacy ``test_reports.json`` file, commits, and puts a
  previously staged artifact back into staging.  It is skipped when the artifact already holds a
  report with the same ``tested_at``.
"""
from __future__ import annotations

import json
import logging
from typing import Any, Awaitable, Callable, Dict, List, Optional

from .. import __version__

logger = logging.getLogger("bioengine.bioimageio")

REPORT_FILE = "test_report.json"
LEGACY_REPORT_FILE = "test_reports.json"
LEGACY_MANIFEST_KEYS = ("test_reports", "test_report", "score")


def implementation_versions() -> Dict[str, str]:
    """Versions of the packages that decide a test's outcome.  The reference pins bioimageio.core /
    bioimageio.spec; here both are implemented in-tree (``bioengine_worker_amd.bioimageio``), so the
    rows carry this framework's version: a framework upgrade invalidates cached reports exactly as a
    bioimageio upgrade does upstream."""
    try:  # an installed upstream package (not in this image) would take precedence
        from importlib.metadata import PackageNotFoundError, version
    except ImportError:  # pragma: no cover
        return {"bioimageio.core": __version__, "bioimageio.spec": __version__}
    out = {}
    for name in ("bioimageio.core", "bioimageio.spec"):
        try:
            out[name] = version(name)
        except PackageNotFoundError:
            out[name] = f"{__version__}+bioengine-amd"
    return out


def env_rows(extra: Optional[Dict[str, str]] = None) -> List[List[str]]:
    rows = [[k, v, "", ""] for k, v in implementation_versions().items()]
    for k, v in (extra or {}).items():
        rows.append([str(k), str(v), "", ""])
    return ensure_bioengine_row({"env": rows})["env"]


def ensure_bioengine_row(report: dict) -> dict:
    """report['env'] as a list of rows with a current ``bioengine`` row (reference :1151-1182).  A
    dict-shaped env (older reports of this framework) is converted to rows."""
    env = report.get("env")
    if isinstance(env, dict):
        env = [[str(k), str(v), "", ""] for k, v in env.items()]
    elif not isinstance(env, list):
        env = []
    else:
        env = [list(r) if isinstance(r, tuple) else r for r in env]
    for i, row in enumerate(env):
        if isinstance(row, list) and row and str(row[0]) == "bioengine":
            row = list(row) + [""] * max(0, 4 - len(row))
            row[1] = __version__
            env[i] = row
            break
    else:
        env.append(["bioengine", __version__, "", ""])
    report["env"] = env
    return report


def cached_report_valid(cached: dict, latest_remote_modified, current: Optional[Dict[str, str]] = None) -> bool:
    """Reuse a cached report only if the package is unchanged AND every implementation version in
    its env matches the installed one (reference :1589-1618)."""
    try:
        if cached["latest_remote_modified"] != latest_remote_modified:
            return False
        report = cached["test_report"]
    except (KeyError, TypeError):
        return False
    current = implementation_versions() if current is None else current
    seen = {}
    for row in report.get("env", []) or []:
        if isinstance(row, (list, tuple)) and len(row) >= 2 and str(row[0]) in current:
            seen[str(row[0])] = str(row[1])
    return all(seen.get(k) == v for k, v in current.items()) and "tested_at" in report


def finalize_report(report: dict, tested_at: float) -> dict:
    report = ensure_bioengine_row(dict(report))
    report["tested_at"] = tested_at
    return report


def fallback_report(model_id: str, source: str, artifact_type, error: str) -> dict:
    """Report of a test run that raised (reference :1670-1697)."""
    v = implementation_versions()
    return {"name": "bioimageio format validation", "source_name": source, "id": model_id, "type": artifact_type,
            "format_version": v.get("bioimageio.spec", "unknown"), "status": "failed",
            "details": [{"errors": [{"msg": error}]}],
            "env": [[k, val, "", ""] for k, val in v.items()], "saved_conda_list": ""}


def _name(f: Any) -> str:
    if isinstance(f, dict):
        return str(f.get("name"))
    return str(getattr(f, "name", f))


async def publish_report(artifact_manager, artifact_id: str, report: dict,
                         http_get: Callable[[str], Awaitable[str]],
                         http_put: Callable[[str, str], Awaitable[None]]) -> str:
    """Publish ``report`` to ``artifact_id``; returns "published" or "up-to-date".

    ``http_get(url) -> text`` / ``http_put(url, text)`` move the file bodies through the presigned
    URLs the artifact manager hands out (httpx in the app, anything in tests)."""
    try:  # skip when the artifact already holds this very report (same tested_at)
        url = await artifact_manager.get_file(artifact_id=artifact_id, file_path=REPORT_FILE)
        remote = json.loads(await http_get(url))
        if float(remote.get("tested_at", 0.0)) == float(report["tested_at"]):
            return "up-to-date"
    except Exception as e:  # noqa: BLE001 -- no remote report yet, or unreadable: publish
        logger.info("no readable remote test report for %s (%s); publishing", artifact_id, e)
    art = await artifact_manager.read(artifact_id=artifact_id)
    was_staged = bool(art.get("staging"))
    manifest = dict(art.get("manifest") or {})
    for k in LEGACY_MANIFEST_KEYS:
        manifest.pop(k, None)
    manifest["test_summary"] = {"status": report["status"], "tested_at": report["tested_at"], "env": report["env"]}
    art = await artifact_manager.edit(artifact_id=art["id"], manifest=manifest, stage=True)
    url = await artifact_manager.put_file(art["id"], file_path=REPORT_FILE)
    await http_put(url, json.dumps(report, default=str))
    try:
        files = await artifact_manager.list_files(art["id"], version="stage")
        if any(_name(f) == LEGACY_REPORT_FILE for f in files):
            await artifact_manager.remove_file(art["id"], file_path=LEGACY_REPORT_FILE)
    except Exception as e:  # noqa: BLE001 -- legacy cleanup is best effort, as upstream
        logger.warning("could not remove the legacy %s of %s: %s", LEGACY_REPORT_FILE, artifact_id, e)
    await artifact_manager.commit(artifact_id=art["id"])
    if was_staged:
        await artifact_manager.edit(artifact_id=art["id"], stage=True)
    return "published"
