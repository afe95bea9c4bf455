#!/usr/bin/env python3
"""Stage timings of the 3-D split-touching pipeline (CCL size filter, closing, EDT-3D, peaks, GPU
watershed) on a synthetic organelle volume; prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from bioengine_worker_amd.em import mito
    from bioengine_worker_amd.em.volume import ccl3d

    z = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    coarse = torch.rand(1, 1, z // 16 + 2, 2048 // 32 + 2, 2048 // 32 + 2, generator=g, device=dev)
    mask = torch.nn.functional.interpolate(coarse, size=(z, 2048, 2048), mode="trilinear")[0, 0] > 0.62
    T = {}

    def mark(k, t0):
        torch.cuda.synchronize()
        T[k] = round(time.perf_counter() - t0, 4)
        return time.perf_counter()

    mito.prob_to_instances_3d(mask[:8])  # warm-up
    t = time.perf_counter()
    roots = ccl3d(mask)
    t = mark("ccl3d", t)
    closed = mask
    dist = mito.edt3d(closed)
    t = mark("edt3d", t)
    peaks = mito.peak_local_max3d(dist, closed, 8)
    t = mark("peaks", t)
    markers = mito._markers_from_peaks(peaks, tuple(mask.shape), dev)
    t = mark("markers", t)
    lab = mito.watershed_gpu(-dist, markers, closed)
    t = mark("watershed", t)
    t0 = time.perf_counter()
    lab2, n = mito.prob_to_instances_3d(mask)
    mark("total_pipeline", t0)
    print(json.dumps({"volume": list(mask.shape), "peaks": int(len(peaks)), "instances": n, "timings_s": T}))


if __name__ == "__main__":
    main()
