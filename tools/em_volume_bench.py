#!/usr/bin/env python3
"""FIB-SEM mitochondria volume analysis throughput (BASELINE config 4: 3-D tiled inference over a synthetic
2048^3 volume, z-slabs sharded across the GPUs of one node, RCCL all-gather of the stitched mask).

Each rank synthesises its own z-slab on its GPU (uint8 EM-like texture with ellipsoidal organelles), then
runs ``em.volume.analyze_volume``: percentile normalisation (all-reduced), slice-wise 512² tiled U-Net
inference (BioImage.IO 2-D U-Net 32-256 through the MI355X graph pass, tiles of several slices per model
call), Gaussian blend, threshold, 6-connected HIP CCL, cross-slab label merge, instance stats all-reduce
and the all-gather of the full mask.  Reports voxels/s for the whole volume (max time over ranks).

1 GPU:  ``python tools/em_volume_bench.py --z 256``  (the per-GPU share of 2048^3 on 8 GPUs)
N GPUs: ``torchrun --nproc-per-node N tools/em_volume_bench.py --z 2048``
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def synthetic_slab(z0: int, z1: int, Y: int, X: int, dev, seed: int = 0) -> torch.Tensor:
    g = torch.Generator(device=dev).manual_seed(seed + z0)
    dz = max(2, (z1 - z0) // 16 + 2)
    coarse = torch.rand(1, 1, dz, Y // 32 + 2, X // 32 + 2, generator=g, device=dev)
    field = torch.nn.functional.interpolate(coarse, size=(z1 - z0, Y, X), mode="trilinear", align_corners=False)[0, 0]
    organelles = (field > 0.62).float()
    tex = torch.rand(z1 - z0, Y, X, generator=g, device=dev)
    return (90 + 80 * organelles + 40 * tex).clamp(0, 255).to(torch.uint8)


def main():
    if os.environ.get("BE_DUMP_STACKS"):  # periodic stack dumps to find where a long run spends its time
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["BE_DUMP_STACKS"]), repeat=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--z", type=int, default=256, help="total volume depth (split across ranks)")
    ap.add_argument("--yx", type=int, default=2048)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--overlap", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32, help="tiles per model call")
    ap.add_argument("--gather", default="mask", choices=["mask", "labels", "rank0", "sharded", "none"],
                    help="mask/labels: all-gather onto every rank; rank0: dist.gather of the label volume onto "
                         "rank 0 only; sharded: labels stay on the rank that computed them")
    ap.add_argument("--split-touching", action="store_true",
                    help="3-D closing + EDT + peaks + GPU marker watershed instead of plain CCL")
    a = ap.parse_args()

    world, rank, local = int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from bioengine_worker_amd.bioimageio.package import write_unet2d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.em.volume import analyze_volume, slab_bounds

    root = Path(tempfile.mkdtemp(prefix=f"em-bench-{rank}-")) / "mito-unet2d"
    write_unet2d_package(root, "mito-unet2d", in_channels=1, out_channels=1, features=(32, 64, 128, 256),
                         test_shape=(1, 1, 128, 128), torchscript=False)
    pipe = PredictionPipeline(root, device=dev)

    def predict(t):
        return next(iter(pipe.predict_tensors(t).values()))

    z0, z1 = slab_bounds(a.z, rank, world)
    slab = synthetic_slab(z0, z1, a.yx, a.yx, dev)
    # warm-up on a few slices (graph pass, kernels, allocator)
    w = analyze_volume(slab[: min(4, z1 - z0)], predict, a.tile, a.overlap, a.batch, timings=True)
    torch.cuda.synchronize()
    if rank == 0:
        print(json.dumps({"warmup_slices": min(4, z1 - z0), "timings_s": w["timings_s"],
                          "n_components": w["n_components"]}), flush=True)
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    res = analyze_volume(slab, predict, a.tile, a.overlap, a.batch, group=None, z_offset=z0,
                         gather=a.gather if a.gather in ("mask", "labels") else None, timings=True,
                         split_touching=a.split_touching)
    if a.gather == "rank0":
        from bioengine_worker_amd.em.volume import gather_to_rank0

        tg = time.perf_counter()
        full = gather_to_rank0(res["labels_slab_t"])
        torch.cuda.synchronize()
        res["timings_s"]["gather_rank0"] = round(time.perf_counter() - tg, 4)
        res["rank0_volume_shape"] = list(full.shape) if full is not None else None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t
    if world > 1:
        d = torch.tensor([dt], device=dev)
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
        dt = float(d)
    if rank == 0:
        vox = a.z * a.yx * a.yx
        print(json.dumps({"metric": "fibsem_volume_voxels_per_sec", "value": round(vox / dt, 1), "unit": "voxel/s",
                          "n_gpus": world, "seconds": round(dt, 3), "volume": [a.z, a.yx, a.yx],
                          "tiles_per_slice": len(range(0, a.yx, a.tile - a.overlap)) ** 2, "tile": a.tile,
                          "overlap": a.overlap, "n_instances": res["n_instances"], "n_components": res["n_components"],
                          "gathered": a.gather, "split_touching": a.split_touching,
                          "timings_s": res["timings_s"], "dtype": "bf16 (graph-pass U-Net)",
                          "data": "synthetic EM-like uint8 volume, random-init U-Net weights"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
