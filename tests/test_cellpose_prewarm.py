"""The Cellpose app's replica start-up runs every continuous-batching size once (largest first), so
the first request batch of each size in traffic pays no one-time allocation / plan cost on the
request path (the round-5 router p99 tail: the first two 32-image batches at c = 64)."""
import asyncio
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
APP_MAIN = ROOT / "apps" / "cellpose-finetuning" / "main.py"


@pytest.mark.unit
def test_async_init_prewarms_every_batch_size(tmp_path, monkeypatch):
    from bioengine_worker_amd.compat import install
    from bioengine_worker_amd.serve.batching import batch_stats

    install()
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.setenv("BE_CELLPOSE_PREWARM", "force")
    monkeypatch.setenv("BE_CELLPOSE_PREWARM_SIZE", "64")
    spec = importlib.util.spec_from_file_location("cellpose_main_prewarm_test", APP_MAIN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cls = mod.CellposeFinetune.func_or_class
    # the default covers every size the batcher can form (max_batch_size 32), largest first
    assert cls.PREWARM_BATCHES == tuple(range(32, 0, -1))
    # the mechanism on a CPU-sized subset (odd sizes included): each runs as one whole batch
    monkeypatch.setattr(cls, "PREWARM_BATCHES", (7, 5, 3, 2, 1))
    app = cls(default_model="cyto3")

    async def main():
        await app.async_init()
        return batch_stats(app, "_segment_batch")

    st = asyncio.run(asyncio.wait_for(main(), 600))
    # every bucket ran as one whole batch before any traffic (the 5 ms window gathers a bucket's
    # concurrent requests into a single batch), the largest first
    assert st is not None and st["requests"] == sum(cls.PREWARM_BATCHES)
    assert {int(k) for k in st["hist"]} == set(cls.PREWARM_BATCHES), st["hist"]
    assert cls.PREWARM_BATCHES[0] == max(cls.PREWARM_BATCHES)
