"""Native host runtime (csrc/runtime): sanitizer builds + the shared-memory ring's Python face.

* ASan+UBSan and TSan builds of every runtime source with the C++ self-test driver
  (``tools/sanitize_runtime.py``; SURVEY.md §5 race detection / sanitizers).
* ``ShmRing`` across two Python processes (spawned child opens the ring by name, echoes frames back
  through a second ring).
"""
import multiprocessing as mp
import os
import shutil
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.parametrize("mode", ["asan", "tsan"])
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_sanitizers(mode, capsys):
    import sanitize_runtime

    rc = sanitize_runtime.run(mode)
    out = capsys.readouterr().out
    assert rc == 0, out
    assert "runtime selftest ok" in out


def _echo(rx_name, tx_name, n):
    sys.path.insert(0, ROOT)
    from bioengine_worker_amd.runtime.shm_ring import ShmRing

    rx, tx = ShmRing.open(rx_name), ShmRing.open(tx_name)
    for _ in range(n):
        a = rx.read(timeout_s=30)
        b = rx.read(timeout_s=30)
        tx.write([b, a])  # swap the two frames of each message


def test_shm_ring_cross_process():
    from bioengine_worker_amd.runtime.shm_ring import RingClosed, ShmRing

    a2b, b2a = ShmRing.create(1 << 20), ShmRing.create(1 << 20)
    p = mp.get_context("spawn").Process(target=_echo, args=(a2b.name, b2a.name, 50))
    p.start()
    rng = np.random.default_rng(0)
    try:
        for i in range(50):
            x = rng.integers(0, 255, size=int(rng.integers(0, 300_000)), dtype=np.uint8)
            y = rng.integers(0, 255, size=17 * i, dtype=np.uint8)
            a2b.write([x, memoryview(y)])
            assert bytes(b2a.read(timeout_s=30)) == y.tobytes()
            assert bytes(b2a.read(timeout_s=30)) == x.tobytes()
    finally:
        p.join(30)
        a2b.unlink()
        b2a.unlink()
    assert p.exitcode == 0
    st = a2b.stats()
    assert st["frames"] == 100 and st["queued_bytes"] == 0
    with pytest.raises(ValueError):
        a2b.write([np.zeros(2 << 20, np.uint8)])
    with pytest.raises(TimeoutError):
        a2b.read(timeout_s=0.01)
    a2b.shutdown()
    with pytest.raises(RingClosed):
        a2b.write([b"x"])


def _echo_big(rx_name, tx_name, n):
    sys.path.insert(0, ROOT)
    from bioengine_worker_amd.runtime.shm_ring import ShmRing, tune_malloc

    tune_malloc()
    rx, tx = ShmRing.open(rx_name), ShmRing.open(tx_name)
    for _ in range(n):
        tx.write([rx.read(timeout_s=30)])


def test_shm_ring_large_frames_cross_process():
    """Frames past the parallel-copy threshold (512 KiB, split over the copy pool's threads in both
    processes), wrapping an 8 MiB ring many times, with the replicas' malloc tuning on."""
    from bioengine_worker_amd.runtime.shm_ring import ShmRing, tune_malloc

    assert tune_malloc()  # default on; idempotent
    a2b, b2a = ShmRing.create(8 << 20), ShmRing.create(8 << 20)
    n = 24
    p = mp.get_context("spawn").Process(target=_echo_big, args=(a2b.name, b2a.name, n))
    p.start()
    rng = np.random.default_rng(1)
    try:
        for i in range(n):
            x = rng.integers(0, 255, size=(512 << 10) + int(rng.integers(0, 3 << 20)), dtype=np.uint8)
            a2b.write([x])
            y = b2a.read(timeout_s=30)
            assert y.nbytes == x.nbytes and np.array_equal(y, x)
    finally:
        p.join(30)
        a2b.unlink()
        b2a.unlink()
    assert p.exitcode == 0


@pytest.mark.parametrize("hw", [(771, 28), (96, 96), (224, 224), (1, 1), (3, 5)])
def test_native_png_roundtrips_through_pil(hw):
    """The host runtime's stored-deflate PNG encoder (csrc/runtime/png.cpp) decodes bit-exactly in
    PIL, including raw sizes that are exact multiples of the 65535-byte block (28 x 771: (3*28+1)*771
    = 65535), where the IDAT length once counted one block too many."""
    import base64
    import io

    from PIL import Image

    from bioengine_worker_amd.search.ingestion import png_b64_batch

    h, w = hw
    rng = np.random.default_rng(h * 1000 + w)
    rgb = rng.integers(0, 256, (3, h, w, 3), dtype=np.uint8)
    for i, s in enumerate(png_b64_batch(rgb)):
        im = Image.open(io.BytesIO(base64.b64decode(s)))
        im.load()
        assert im.size == (w, h) and im.mode == "RGB"
        assert np.array_equal(np.asarray(im), rgb[i])


def test_native_b64decode_matches_stdlib():
    import base64

    from bioengine_worker_amd.search.ingestion import b64decode_batch

    rng = np.random.default_rng(7)
    payloads = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (0, 1, 2, 3, 4, 5, 63, 64, 65, 1000, 65537)]
    enc = [base64.b64encode(p).decode() for p in payloads]
    for p, got in zip(payloads, b64decode_batch(enc)):
        assert bytes(got) == p
    # one malformed string yields None in its own slot only
    got = b64decode_batch([enc[9], "abc", enc[10]])
    assert bytes(got[0]) == payloads[9] and bytes(got[2]) == payloads[10]
    assert got[1] is None or bytes(got[1]) != b""
