"""Chrome-trace export of request / router / pipeline spans."""
import asyncio
import json

import numpy as np

from bioengine_worker_amd.profiling import trace


def test_trace_spans_and_export(tmp_path):
    trace.clear()
    trace.enable(True)
    try:
        from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, synthetic_cells
        from bioengine_worker_amd.models.cpnet import CPnet

        r = CellposeRunner(CPnet(nbase=[2, 8, 16, 32, 64]).randomize_(0), "cpu")
        with trace.request("eval"):
            r.eval(synthetic_cells(1, 64, 64, ncells=4), tile=False)

        async def serve_calls():
            from bioengine_worker_amd.serve import api as serve
            from bioengine_worker_amd.serve.controller import ServeController, set_controller

            set_controller(ServeController(tick_s=0.05))

            @serve.deployment(num_replicas=1)
            class Echo:
                def ping(self, x):
                    return x

            h = await serve.run(Echo.bind(), name="tr")
            for i in range(3):
                assert await h.ping.remote(i) == i
            await serve.delete("tr")

        asyncio.run(serve_calls())
        doc = trace.export(str(tmp_path / "t.json"))
        names = {e["name"] for e in doc["traceEvents"]}
        assert {"eval", "cellpose.normalize99", "cellpose.masks", "router.admission", "replica.ping"} <= names
        reqs = {e["args"].get("req") for e in doc["traceEvents"] if e["name"].startswith("cellpose.")}
        assert len(reqs) == 1 and None not in reqs
        json.loads((tmp_path / "t.json").read_text())
        s = trace.summary()
        assert s["replica:replica.ping"]["count"] == 3
    finally:
        trace.enable(False)
        trace.clear()
