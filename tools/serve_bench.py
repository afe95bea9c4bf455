#!/usr/bin/env python3
"""End-to-end serving benchmark: Cellpose inference requests through the whole worker stack.

client --(hub RPC)--> app service --> router (admission, deadlines) --> GPU-pinned process replica
(shared-memory ring for the image/mask payloads) --> ``@serve.batch`` continuous batching -->
HIP CPnet + dynamics + masks --> back.

Each client sends ONE 512x512 2-channel image per request (the reference's cellpose service handles
one request at a time per replica, ``apps/cellpose-finetuning/main.py:3616-3623``); C clients run
closed-loop.  Reports img/s and p50/p95/p99 request latency per concurrency level.
Usage: ``python tools/serve_bench.py [--size 512] [--concurrency 1,8,32] [--seconds 10] [--gpus 1]``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402


async def main_async(a) -> list[dict]:
    from bioengine_worker_amd.cellpose.pipeline import synthetic_cells
    from bioengine_worker_amd.transport import connect_to_server
    from bioengine_worker_amd.transport.hub import get_local_hub
    from bioengine_worker_amd.worker.worker import BioEngineWorker

    os.environ.setdefault("BIOENGINE_LOCAL_ARTIFACT_PATH", str(ROOT / "apps"))
    os.environ.setdefault("BIOENGINE_REPLICA_MODE", a.replica_mode)
    tmp = Path(tempfile.mkdtemp(prefix="serve-bench-"))
    os.environ["HOME"] = str(tmp / "home")
    hub = get_local_hub("sbench")
    await hub.start_http()
    tok = hub.issue_token("admin-user", workspace="ws-admin")
    w = BioEngineWorker(mode="single-machine", workspace_dir=tmp / "be", server_url="local://sbench", token=tok,
                        client_id="worker1", log_file="off", head_num_cpus=8, head_num_gpus=a.gpus,
                        monitoring_interval_seconds=5, data_server_url=None)
    await w.start(blocking=False)
    admin = await connect_to_server({"server_url": "local://sbench", "token": tok})
    svc = await admin.get_service(w.full_service_id)
    # deploy_app's max_ongoing_requests (the app proxy's cap, default 10 as in the reference) bounds
    # how many requests can reach the replica's batcher at once
    aid = await svc.deploy_app(artifact_id="cellpose-finetuning", application_id="cpbench", disable_gpu=a.gpus == 0,
                               max_ongoing_requests=a.max_ongoing, hypha_token=tok,
                               application_kwargs={"CellposeFinetune": {"default_model": a.model}})
    st = await w.apps_manager.wait_for(aid, timeout=600)
    assert st == "RUNNING", (await svc.get_app_status(application_ids=[aid]))["message"]
    s = await svc.get_app_status(application_ids=[aid])
    app = await admin.get_service(s["service_ids"][0]["websocket_service_id"])
    imgs = [synthetic_cells(1, a.size, a.size, ncells=60, seed=i)[0] for i in range(16)]
    for i in range(3):  # warm-up: model build, kernels, graph pass, batch shapes
        await asyncio.gather(*[app.infer(input_arrays=[imgs[j % 16]], model=a.model) for j in range(8)])
    results = []
    if getattr(a, "layer", "hub") == "handle":  # bypass the hub RPC + app-service bridge: router -> replica only
        handle = w.apps_manager.apps[aid]["bridge"].handle

        class _H:
            async def infer(self, **kw):
                return await handle.infer.remote(**kw)

        app = _H()
    timeline = getattr(a, "timeline", None)
    gc_events: list = []
    if timeline:  # GC pauses of this process (hub + worker + router + clients share its event loop)
        import gc

        _gc_t0 = {}

        def _gc_cb(phase, info):
            if phase == "start":
                _gc_t0["t"] = time.perf_counter()
            else:
                gc_events.append((_gc_t0.get("t", 0.0), time.perf_counter() - _gc_t0.get("t", 0.0), info["generation"],
                                  info["collected"]))

        gc.callbacks.append(_gc_cb)
    for conc in a.concurrency:
        lat: list[float] = []
        starts: list[float] = []
        # Closed-loop ramp: all `conc` clients fire at once when a level starts, so its first requests
        # queue behind each other (at c = 64 two 32-image batches: ~37 and ~52 ms against a ~30 ms
        # steady state).  Requests STARTED in the first `ramp` seconds are reported separately
        # (ramp_requests / ramp_max_ms / p99_ms_incl_ramp), the percentiles and rate are over the
        # `seconds` window after it.
        ramp = float(getattr(a, "ramp", 0.5) or 0.0)
        stop = time.perf_counter() + ramp + a.seconds

        async def client(cid):
            k = cid
            while time.perf_counter() < stop:
                t = time.perf_counter()
                out = await app.infer(input_arrays=[imgs[k % 16]], model=a.model)
                lat.append(time.perf_counter() - t)
                starts.append(t)
                assert out[0]["output"].shape == (a.size, a.size)
                k += conc

        prof = None
        if a.profile and conc == max(a.concurrency):
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        await asyncio.gather(*[client(c) for c in range(conc)])
        dt = time.perf_counter() - t0
        if prof is not None:
            import io
            import pstats

            prof.disable()
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
            pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(120)
            Path(a.profile).write_text(buf.getvalue())
        ms_all = np.array(lat) * 1e3
        keep = np.array(starts) >= t0 + ramp
        ms = ms_all[keep] if keep.any() else ms_all
        n_win = int(keep.sum()) if keep.any() else len(lat)
        win = a.seconds if keep.any() else dt
        if timeline:
            thr = float(np.percentile(ms, 99))
            slow = sorted((round(st - t0, 4), round(l * 1e3, 2)) for st, l in zip(starts, lat) if l * 1e3 >= thr)
            gcs = [(round(t - t0, 4), round(d * 1e3, 2), g, c) for t, d, g, c in gc_events if t >= t0 and d > 0.002]
            with open(timeline, "a") as fh:
                fh.write(json.dumps({"concurrency": conc, "phase_s": round(dt, 3), "p99_ms": round(thr, 2),
                                     "slow_start_s_and_ms": slow[:200], "gc_pauses_over_2ms_s_ms_gen_collected": gcs})
                         + "\n")
        r = {"concurrency": conc, "requests": n_win, "imgs_per_s": round(n_win / win, 1),
             "p50_ms": round(float(np.percentile(ms, 50)), 2), "p95_ms": round(float(np.percentile(ms, 95)), 2),
             "p99_ms": round(float(np.percentile(ms, 99)), 2), "ramp_s": ramp, "ramp_requests": len(lat) - n_win,
             "ramp_max_ms": round(float(ms_all[~keep].max()), 2) if (~keep).any() else None,
             "p99_ms_incl_ramp": round(float(np.percentile(ms_all, 99)), 2), "image": [a.size, a.size, 2], "gpus": a.gpus,
             "replica_mode": os.environ["BIOENGINE_REPLICA_MODE"], "layer": getattr(a, "layer", "hub")}
        results.append(r)
        print(json.dumps(r), flush=True)
    st = await svc.get_app_status(application_ids=[aid])
    print(json.dumps({"router": {k: v.get("latency_ms") for k, v in st.get("deployments", {}).items()}}), flush=True)
    try:
        print(json.dumps({"batching": await app.get_batch_stats()}), flush=True)
    except Exception:  # noqa: BLE001
        pass
    await svc.stop_app(application_id=aid)
    await w._cleanup()
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--concurrency", default="1,8,32")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--replica-mode", default="process", choices=["process", "local"])
    ap.add_argument("--max-ongoing", type=int, default=64, help="deploy_app max_ongoing_requests")
    ap.add_argument("--layer", default="hub", choices=["hub", "handle"],
                    help="hub: client -> hub RPC -> app service -> router (default); handle: router directly")
    ap.add_argument("--model", default="cyto3", help="built-in model served (headline: cyto3 CPnet)")
    ap.add_argument("--ramp", type=float, default=0.5,
                    help="seconds at the start of each concurrency level whose requests are reported separately")
    ap.add_argument("--timeline", default=None, metavar="PATH",
                    help="append, per concurrency level, the start times of the requests at or above p99 and the "
                         "GC pauses (> 2 ms) of the benchmark process")
    ap.add_argument("--profile", default=None, metavar="PATH",
                    help="cProfile the worker-side event loop during the highest-concurrency phase")
    a = ap.parse_args()
    a.concurrency = [int(c) for c in a.concurrency.split(",")]
    asyncio.run(main_async(a))


if __name__ == "__main__":
    main()
