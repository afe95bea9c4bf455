#!/usr/bin/env python3
"""Served cell-image-search queries through the whole worker stack (BASELINE config 5: "batched
-request serving path").

client --(hub RPC)--> app service --> router --> GPU process replica --> ``@serve.batch`` query
embedding (fp8 DINOv2 ViT-B/14, up to 64 per forward) --> ``@serve.batch`` index scan --> back.

Each client sends ONE 224x224x3 crop per request (``search(image_b64=...)``, top-20) closed-loop;
C clients.  The index is a synthetic Cell-Painting dataset ingested by the app itself.  Reports
queries/s and p50/p95/p99 per concurrency, plus the app's batch histogram.
Usage: ``python tools/search_serve_bench.py [--concurrency 1,64] [--seconds 5]``.
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import io
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402


def _batch_delta(before: dict, after: dict) -> float | None:
    """Mean query batch over one concurrency level (the app's counters are cumulative)."""
    nb = after.get("batches", 0) - before.get("batches", 0)
    return round((after.get("requests", 0) - before.get("requests", 0)) / nb, 2) if nb else None


async def main_async(a) -> list[dict]:
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    os.environ.setdefault("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    os.environ.setdefault("BIOENGINE_REPLICA_MODE", a.replica_mode)
    tmp = Path(tempfile.mkdtemp(prefix="search-bench-"))
    os.environ["HOME"] = str(tmp / "home")
    hub = get_local_hub("qbench")
    await hub.start_http()
    tok = hub.issue_token("admin-user", workspace="ws-admin")
    w = BioEngineWorker(mode="single-machine", workspace_dir=tmp / "be", server_url="local://qbench", token=tok,
                        client_id="worker1", log_file="off", head_num_cpus=8, head_num_gpus=a.gpus,
                        monitoring_interval_seconds=5, data_server_url=None)
    await w.start(blocking=False)
    admin = await connect_to_server({"server_url": "local://qbench", "token": tok})
    svc = await admin.get_service(w.full_service_id)
    aid = await svc.deploy_app(artifact_id="cell-image-search", application_id="qbench", disable_gpu=a.gpus == 0,
                               max_ongoing_requests=a.max_ongoing,
                               application_kwargs={"CellImageSearch": {"model": a.model}})
    st = await w.apps_manager.wait_for(aid, timeout=600)
    assert st == "RUNNING", (await svc.get_app_status(application_ids=[aid]))["message"]
    s = await svc.get_app_status(application_ids=[aid])
    app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])
    r = await app.add_synthetic_dataset(n_images=a.n_images, n_crops_per_image=40)
    for _ in range(3000):
        ist = await app.get_ingestion_status(session_id=r["session_id"])
        if ist["status"] in ("completed", "failed", "stopped"):
            break
        await asyncio.sleep(0.1)
    assert ist["status"] == "completed", ist
    n_cells = (await app.get_index_stats())["n_cells"]
    rng = np.random.default_rng(0)
    crops = []
    for i in range(16):
        buf = io.BytesIO()
        np.save(buf, (rng.random((224, 224, 3)) * 255).astype(np.uint8))
        crops.append(base64.b64encode(buf.getvalue()).decode())
    for _ in range(3):  # warm-up: engine, batch shapes
        await asyncio.gather(*[app.search(image_b64=crops[j % 16], top_k=20) for j in range(16)])
    results = []
    for conc in a.concurrency:
        lat: list[float] = []
        srv: list[float] = []
        last: dict = {}
        q0 = (await app.get_batch_stats()).get("query", {})
        stop = time.perf_counter() + a.seconds

        async def client(cid):
            k = cid
            while time.perf_counter() < stop:
                t = time.perf_counter()
                out = await app.search(image_b64=crops[k % 16], top_k=20)
                lat.append(time.perf_counter() - t)
                srv.append(out.get("elapsed_ms", 0.0))
                last["o"] = out
                assert len(out["results"]) == min(20, n_cells)
                k += conc

        prof = None
        if getattr(a, "profile", None) and conc == max(a.concurrency):
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        await asyncio.gather(*[client(c) for c in range(conc)])
        dt = time.perf_counter() - t0
        if prof is not None:
            import io as _io
            import pstats

            prof.disable()
            buf = _io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
            pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(80)
            Path(a.profile).write_text(buf.getvalue())
        ms = np.array(lat) * 1e3
        rr = {"concurrency": conc, "requests": len(lat), "qps": round(len(lat) / dt, 1),
              "p50_ms": round(float(np.percentile(ms, 50)), 2), "p95_ms": round(float(np.percentile(ms, 95)), 2),
              "p99_ms": round(float(np.percentile(ms, 99)), 2), "n_cells": n_cells, "model": a.model,
              "replica_p50_ms": round(float(np.percentile(srv, 50)), 2),
              "mean_query_batch": _batch_delta(q0, (await app.get_batch_stats()).get("query", {})),
              "response_kb": round(len(json.dumps(last.get("o", {}))) / 1024, 1)}
        results.append(rr)
        print(json.dumps(rr), flush=True)
    bs = await app.get_batch_stats()
    print(json.dumps({"batching": bs}), flush=True)
    for rr in results:
        rr["batching"] = bs.get("query", {})
    await svc.stop_app(application_id=aid)
    await w._cleanup()
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", default="1,64")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--n-images", type=int, default=4)
    ap.add_argument("--model", default="vitb14")
    ap.add_argument("--max-ongoing", type=int, default=64)
    ap.add_argument("--replica-mode", default="process")
    ap.add_argument("--profile", default=None, metavar="PATH",
                    help="cProfile of this process (client + hub + bridge + router) at the highest concurrency")
    a = ap.parse_args()
    a.concurrency = [int(c) for c in a.concurrency.split(",")]
    asyncio.run(main_async(a))


if __name__ == "__main__":
    main()
