"""Garbage-collector policy for latency-sensitive serving processes.

CPython's cyclic GC walks every tracked container of a generation when its allocation counter
trips; a full (generation 2) pass over a serving process -- worker + router + hub, or a replica with
its app state, model wrappers and imported torch modules -- is tens of milliseconds, and it runs on
the event-loop thread in the middle of whichever request triggered it.  At 64 concurrent clients
those pauses land in the latency tail (profiles/r03/serve_*).

Policy (``BIOENGINE_GC_TUNE=0`` disables it): collect once, then ``gc.freeze()`` the surviving
startup objects into the permanent generation so later scans skip them, and raise the young-
generation threshold so request garbage is collected in fewer, cheaper passes.  Objects created
by lazy app initialisation are frozen again by :func:`refreeze` once the app reports healthy.
"""
from __future__ import annotations

import gc
import os

_done = False


def enabled() -> bool:
    return os.environ.get("BIOENGINE_GC_TUNE", "1") != "0"


def serving_gc(threshold0: int = 50_000) -> None:
    global _done
    if not enabled():
        return
    gc.collect()
    gc.freeze()
    t = gc.get_threshold()
    gc.set_threshold(max(t[0], threshold0), max(t[1], 20), max(t[2], 50))
    _done = True


def refreeze() -> None:
    """Move everything alive now (e.g. a model built by ``async_init``) out of the collector's scans."""
    if enabled() and _done:
        gc.collect(1)
        gc.freeze()
