#!/usr/bin/env python3
"""Upload an application directory (manifest.yaml + Python files + assets) as an app artifact.

    python scripts/upload_app.py apps/demo-app --server-url https://hypha.aicell.io --workspace my-ws
    python scripts/upload_app.py apps/cellpose-finetuning --server-url ws://127.0.0.1:9527 --token $HYPHA_TOKEN

Talks to the hub's ``public/artifact-manager`` directly (no worker needed): stages the artifact in
``<workspace>/applications``, uploads every file, prunes files that disappeared from the directory
and commits (a new version tag when the manifest version changed).  ``--dry-run`` only validates
the manifest and lists what would be uploaded.  Reference: scripts/upload_app.py (17-194).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from bioengine_worker_amd.utils.artifact_utils import (  # noqa: E402
    create_application_from_files,
    create_file_list_from_directory,
    load_manifest_from_files,
    validate_manifest,
)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("app_dir", type=Path)
    ap.add_argument("--server-url", default=os.environ.get("BIOENGINE_SERVER_URL", "https://hypha.aicell.io"))
    ap.add_argument("--workspace", default=os.environ.get("HYPHA_WORKSPACE"))
    ap.add_argument("--token", default=os.environ.get("HYPHA_TOKEN") or os.environ.get("BIOENGINE_TOKEN"))
    ap.add_argument("--artifact-id-suffix", default=None, help="append '-SUFFIX' to the manifest id (test uploads)")
    ap.add_argument("--dry-run", action="store_true")
    return ap.parse_args(argv)


async def upload(args) -> str:
    from bioengine_worker_amd.transport import connect_to_server

    files = create_file_list_from_directory(args.app_dir, args.artifact_id_suffix)
    cfg = {"server_url": args.server_url}
    if args.token:
        cfg["token"] = args.token
    if args.workspace:
        cfg["workspace"] = args.workspace
    server = await connect_to_server(cfg)
    try:
        am = await server.get_service("public/artifact-manager")
        ws = args.workspace or server.config.workspace
        return await create_application_from_files(am, files, ws)
    finally:
        try:
            await server.disconnect()
        except Exception:  # noqa: BLE001
            pass


def main(argv=None) -> int:
    args = parse_args(argv)
    files = create_file_list_from_directory(args.app_dir, args.artifact_id_suffix)
    manifest = load_manifest_from_files(files)
    validate_manifest(manifest)
    if args.dry_run:
        print(json.dumps({"id": manifest["id"], "version": manifest.get("version"),
                          "files": [f["name"] for f in files]}, indent=2))
        return 0
    aid = asyncio.run(upload(args))
    print(f"uploaded {args.app_dir} -> {aid}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
