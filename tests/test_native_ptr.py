"""ops/_native.ptr keeps the tensor it points at alive for the duration of the call, so converted
temporaries in one argument list never share a caching-allocator block (the IVF scan once read its
query block overwritten by the probe indices converted right after it)."""
import ctypes
import gc

import torch


def test_ptr_keeps_temporaries_alive():
    from bioengine_worker_amd.ops import _native

    ps = [_native.ptr(torch.full((1024,), float(i)) * 2) for i in range(4)]  # temporaries only
    gc.collect()
    addrs = {p.value for p in ps}
    assert len(addrs) == 4  # four live, distinct blocks
    for i, p in enumerate(ps):
        assert isinstance(p, ctypes.c_void_p)
        vals = (ctypes.c_float * 1024).from_address(p.value)
        assert vals[0] == 2.0 * i and vals[1023] == 2.0 * i
    assert _native.ptr(None) is None
