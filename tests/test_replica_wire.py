"""Process-replica message framing (serve/replica.py): long strings (base64 images / thumbnails)
leave the pickle header as out-of-band UTF-8 buffers -- so they ride the shared-memory ring with the
arrays -- and come back equal, with no copy of the message skeleton when nothing qualifies."""
import numpy as np

from bioengine_worker_amd.serve import replica as rp


def test_long_strings_out_of_band_roundtrip():
    obj = ("resp", 3, {"results": [{"rank": i, "thumbnail_b64": "A" * 20000, "s": 0.5} for i in range(20)],
                       "query_thumbnail_b64": "é" * 100000, "small": "x", "tup": ("C" * rp.BIG_STR, 7)})
    frames = rp.dumps(obj)
    assert len(frames) == 1 + 22 and len(frames[0]) < 4096
    back = rp.loads([frames[0]] + [np.frombuffer(bytes(f), np.uint8).copy() for f in frames[1:]])
    assert back == obj


def test_small_messages_untouched():
    obj = {"a": ["x" * 100, 1, (2.0, "y")], "arr": np.arange(5)}
    assert rp._lift_strings(obj) is obj
    frames = rp.dumps(obj)
    back = rp.loads(frames)
    assert back["a"] == obj["a"] and (back["arr"] == obj["arr"]).all()
