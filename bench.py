#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): Cellpose-cyto3 512x512 imgs/sec (node) + p50 latency;
fine-tune samples/sec.

``python bench.py --gpus N --steps K --warmup W`` — for N > 1 the driver launches one rank per GPU
with ``torch.distributed.run`` (RCCL).  Each rank runs the *full* Cellpose inference pipeline on a
batch of synthetic 512x512 2-channel uint16 images per step (percentile normalisation, 224-tile
gather, CPnet forward on the fused HIP conv kernels, tapered blend, flow following, seed
histogram/expansion, flow-error QC, hole filling) — nothing is skipped inside the timed region.
Work per GPU is fixed as N grows (weak scaling: every GPU is an independent serving replica, the
reference's scaling model — Ray Serve replicas, ``apps/model-runner/runtime_deployment.py:40-50``).

After the timed inference steps, the same process measures (untimed for the headline):
  * p50 / p95 latency of single-image requests (batch 1, direct call),
  * ``imgs_per_sec_cell_like``: the same pipeline with cell-like network outputs (~150 masks per
    image), so the mask stage does realistic work,
  * ``served_*``: continuous-batched serving through the full worker stack (hub RPC, router, GPU
    process replica, ``@serve.batch``), one 512x512 image per request at 1 and 64 clients — BASELINE
    config 2's "continuous-batched" p50 and throughput,
  * fine-tune samples/s: CPnet fwd+bwd + fused AdamW on 256x256 crops, and Cellpose-SAM (ViT-L/8,
    the reference app's model) on the HIP training engine, data-parallel over RCCL when N > 1
    (bucketed, overlapped with backward) — BASELINE config 3,
and reports them as extra fields of the one JSON line rank 0 prints.

The reference publishes no number for these metrics, so ``vs_baseline`` is null;
``vs_reference_algorithm`` is the speedup over the same pipeline with the network run by PyTorch
eager bf16 (MIOpen) — the "reference-algorithm baseline" of BASELINE.md — measured in-process.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
import warnings
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _dist_setup(ngpus: int):
    """One rank per GPU over RCCL.  Rehearsal knobs (never set by the driver): BE_BENCH_BACKEND=gloo
    and BE_BENCH_SHARED_GPU=1 run the N-rank code paths as N processes on ONE GPU over gloo, so the
    multi-rank lines can be exercised on a one-GPU box (timings are meaningless there)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BE_BENCH_SHARED_GPU") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        backend = os.environ.get("BE_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


_STAGE = {"name": "start", "t0": time.time()}


def _progress(stage: str, rank: int = 0) -> None:
    """One stderr line per bench section (and a heartbeat thread repeating the current one every
    60 s): a long multi-rank run shows where it is, and a native crash names its section."""
    _STAGE["name"] = stage
    print(f"[bench r{rank} +{time.time() - _STAGE['t0']:.0f}s] {stage}", file=sys.stderr, flush=True)
    if not _STAGE.get("hb"):
        import threading

        def beat():
            while True:
                time.sleep(60)
                print(f"[bench r{rank} +{time.time() - _STAGE['t0']:.0f}s] ... {_STAGE['name']}", file=sys.stderr,
                      flush=True)

        _STAGE["hb"] = threading.Thread(target=beat, daemon=True)
        _STAGE["hb"].start()


def _barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def _max_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    t = torch.tensor([v], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_infer(args, world, rank, dev):
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells

    runner = CellposeRunner(device=dev, seed=0)
    imgs = torch.from_numpy(synthetic_cells(args.batch, 512, 512, nchan=2, seed=rank)).to(dev)
    p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15,
                   pipeline_chunks=getattr(args, "chunks", 1))
    for _ in range(args.warmup):
        masks, _, _ = runner.eval(imgs, p)
    extra = {}
    if getattr(args, "sequential", False) or args.chunks > 1:
        _barrier(world)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            masks, flows, _ = runner.eval(imgs, p)
        _barrier(world)
        dt = time.perf_counter() - t0
    else:
        # cross-batch pipeline (CellposeRunner.stream): batch i+1's network overlaps batch i's mask
        # recovery on a second stream; every step is still one full batch through the whole
        # pipeline, and the timed region ends after the last batch's masks
        st = runner.stream(p)
        for _ in range(2):
            st.submit(imgs)
        st.flush()
        _barrier(world)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            st.submit(imgs)
        masks, flows, _ = st.flush()
        _barrier(world)
        dt = time.perf_counter() - t0
        # the same batches one eval() at a time (no overlap between consecutive batches)
        _barrier(world)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            m1, _, _ = runner.eval(imgs, p)
        _barrier(world)
        dt_seq = _max_over_ranks(time.perf_counter() - t1, world)
        extra["imgs_per_sec_sequential_batches"] = round(args.batch * args.steps * world / dt_seq, 2)
        extra["pipelined_masks_match_sequential"] = bool(torch.equal(m1, masks))
    dt = _max_over_ranks(dt, world)
    extra.update({"masks_per_image": float(masks.amax(dim=(1, 2)).float().mean().item()),
                  "fg_fraction": float((flows[:, 2] > 0).float().mean().item())})
    if getattr(args, "trace", None) and rank == 0:  # outside the timed region
        from bioengine_worker_amd.profiling import trace

        trace.clear()
        trace.enable(True)
        with trace.request("bench.step", images=args.batch):
            runner.eval(imgs, p)
        torch.cuda.synchronize()
        trace.export(args.trace)
        extra["trace_summary"] = trace.summary()
        trace.enable(False)
    return dt, runner, imgs, p, extra


def bench_latency(runner, imgs, p, n=20):
    one = imgs[:1]
    for _ in range(3):
        runner.eval(one, p)
    torch.cuda.synchronize()
    lat = []
    for _ in range(n):
        t = time.perf_counter()
        runner.eval(one, p)
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    return statistics.median(lat), lat[int(0.95 * (len(lat) - 1))]


def bench_reference_algorithm(runner, imgs, p, steps=3):
    """Same pipeline, network replaced by PyTorch eager bf16 autocast (MIOpen convs)."""
    from bioengine_worker_amd.cellpose.gpu import compute_masks_gpu, normalize99

    net = runner.net.to(imgs.device).to(memory_format=torch.channels_last)
    plan = runner._plan(512, 512, p)

    def run():
        x = normalize99(imgs.float())
        tiles = plan.gather(x, runner.cin_pad)[..., : runner.nchan].permute(0, 3, 1, 2).float()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            yt = net(tiles.contiguous(memory_format=torch.channels_last))[0]
        y = plan.blend(yt.float().contiguous(), imgs.shape[0])
        return compute_masks_gpu(y)

    for _ in range(3):  # MIOpen picks/compiles its conv solutions on the first calls of a fresh box
        run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    runner.net.cpu()
    return (time.perf_counter() - t) / steps


def bench_mask_recovery(dev, batch, steps=3):
    """Mask recovery alone on *cell-like* flows (random-init weights give no convergent flows, so the
    headline run under-exercises seeds/QC/fill): flows from ~150 synthetic cells per 512x512 image."""
    from bioengine_worker_amd.cellpose.gpu import compute_masks_gpu
    from bioengine_worker_amd.train.cellpose_train import labels_to_flows, synthetic_instances

    _, labels = synthetic_instances(batch, 512, 512, ncells=150, seed=7)
    lab = torch.from_numpy(labels).to(dev)
    t = labels_to_flows(lab)
    y = torch.cat([5.0 * t[:, 1:3], torch.where(lab[:, None] > 0, 5.0, -5.0)], 1).contiguous()
    m = compute_masks_gpu(y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m = compute_masks_gpu(y)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dt / batch * 1e3, float(m.amax(dim=(1, 2)).float().mean().item())


def bench_cell_like(runner, imgs, p, steps=3):
    """The timed inference pipeline with the network's output replaced by CELL-LIKE flows (~150
    cells per 512x512 image), so seeding, flow QC and hole filling do realistic work: random-init
    weights give no convergent flows and leave the mask stage nearly idle in the headline run."""
    from bioengine_worker_amd.train.cellpose_train import labels_to_flows, synthetic_instances

    B = imgs.shape[0]
    _, labels = synthetic_instances(B, 512, 512, ncells=150, seed=11)
    lab = torch.from_numpy(labels).to(imgs.device)
    t = labels_to_flows(lab)
    y_cell = torch.cat([5.0 * t[:, 1:3], torch.where(lab[:, None] > 0, 5.0, -5.0)], 1).contiguous()
    x = imgs.float()

    def run():
        y, _, rescale = runner._net_stage(x, p)  # normalise + tiles + CPnet + blend (real work)
        y = y_cell if y.shape == y_cell.shape else y
        return runner.compute_masks(y, p, rescale)

    for _ in range(2):
        m = run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return B / dt, float(m.amax(dim=(1, 2)).float().mean().item())


def bench_served(seconds: float = 4.0, concurrency=(1, 64)) -> dict:
    """Requests through the full serving stack (tools/serve_bench.py): hub RPC -> app service ->
    router -> GPU-pinned process replica (shared-memory ring) -> @serve.batch continuous batching ->
    HIP pipeline -> back; one 512x512 image per request, H2D/D2H inside every request.  Each
    concurrency level runs a 0.5 s ramp (all clients fire at once) before its measured window; the
    ramp's requests are reported as served_ramp_requests_c* and folded into served_p99_ms_c*_incl_ramp."""
    import argparse as _ap
    import asyncio

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import serve_bench

    # BE_SERVE_TIMELINE=PATH: per level, the start times of the requests at or above p99 and this
    # process's GC pauses (tools/serve_bench.py --timeline)
    a = _ap.Namespace(size=512, concurrency=list(concurrency), seconds=seconds, gpus=1, replica_mode="process",
                      max_ongoing=64, model="cyto3", profile=None, timeline=os.environ.get("BE_SERVE_TIMELINE"))
    res = asyncio.run(serve_bench.main_async(a))
    out = {}
    for r in res:
        c = r["concurrency"]
        out[f"served_imgs_per_sec_c{c}"] = r["imgs_per_s"]
        out[f"served_p50_ms_c{c}"] = r["p50_ms"]
        out[f"served_p95_ms_c{c}"] = r["p95_ms"]
        out[f"served_p99_ms_c{c}"] = r["p99_ms"]
        out[f"served_p99_ms_c{c}_incl_ramp"] = r.get("p99_ms_incl_ramp")
        out[f"served_ramp_requests_c{c}"] = r.get("ramp_requests")
    return out


def bench_served_node(args, world: int, rank: int) -> dict:
    """Node-level serving at world > 1: after the per-rank lines every rank frees
    its cached HBM and waits on a host-side (gloo) barrier; rank 0 then deploys the Cellpose app
    through the worker stack with one process replica per GPU (HIP_VISIBLE_DEVICES-pinned children,
    nothing re-execs a GPU process) and drives c = 64 x N closed-loop clients, so the router fans the
    requests out over the node -- the reference's replica scaling
    (bioengine/apps/proxy_deployment.py:35-44, apps/model-runner/runtime_deployment.py:40-50)."""
    import argparse as _ap
    import asyncio
    import gc

    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    gl = dist.new_group(backend="gloo")
    dist.barrier(group=gl)
    out = {}
    if rank == 0:
        try:
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
            import serve_bench

            nrep = max(1, min(world, torch.cuda.device_count()))
            os.environ["BIOENGINE_CELLPOSE_REPLICAS"] = str(nrep)
            os.environ["BIOENGINE_GPU_IDS"] = ",".join(str(i) for i in range(nrep))
            conc = 64 * world
            a = _ap.Namespace(size=512, concurrency=[conc], seconds=max(4.0, 2 * args.served_seconds), gpus=nrep,
                              replica_mode="process", max_ongoing=conc, model="cyto3", profile=None)
            r = asyncio.run(serve_bench.main_async(a))[-1]
            out[f"served_imgs_per_sec_node_c{conc}"] = r["imgs_per_s"]
            out[f"served_p50_ms_node_c{conc}"] = r["p50_ms"]
            out[f"served_p99_ms_node_c{conc}"] = r["p99_ms"]
            out["served_node_config"] = {"replicas": nrep, "gpus_per_replica": 1, "replica_mode": "process",
                                         "clients": conc, "image": [512, 512, 2], "layer": "hub -> router -> replicas"}
        except Exception as e:  # noqa: BLE001
            out["extras_error_served_node"] = f"{type(e).__name__}: {e}"
    dist.barrier(group=gl)
    return out


def bench_vit_embed(dev, batch: int = 64, steps: int = 20) -> float:
    """DINOv2 ViT-B/14 embedding throughput, fp8 e4m3 GEMMs, batch 64 of 224x224 (the reference's
    embedder batch and resolution, apps/cell-image-search/embedder.py:59-95; ~500 img/s/A100 fp16)."""
    from bioengine_worker_amd.search.ingestion import default_engine_factory

    eng = default_engine_factory(dev, "vitb14")
    x = torch.randn(batch, 3, 224, 224, device=dev)
    for _ in range(3):
        eng.embed(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.embed(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    del eng
    torch.cuda.empty_cache()
    return batch / dt


def bench_served_search(seconds: float = 4.0) -> dict:
    """cell-image-search queries through the serving stack (tools/search_serve_bench.py)."""
    import argparse as _ap
    import asyncio

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import search_serve_bench

    a = _ap.Namespace(concurrency=[1, 64], seconds=seconds, gpus=1, n_images=4, model="vitb14", max_ongoing=64,
                      replica_mode="process")
    out, b = {}, {}
    for r in asyncio.run(search_serve_bench.main_async(a)):
        c = r["concurrency"]
        out[f"search_served_qps_c{c}"] = r["qps"]
        out[f"search_served_p50_ms_c{c}"] = r["p50_ms"]
        out[f"search_served_p99_ms_c{c}"] = r["p99_ms"]
        out[f"search_served_mean_batch_c{c}"] = r.get("mean_query_batch")
        b = r.get("batching") or {}
    if b:  # the app's query batcher over the whole run (all concurrency levels)
        out["search_served_query_batching"] = {k: b[k] for k in ("batches", "requests", "mean_batch", "hist") if k in b}
    return out


def bench_em_volume(args, world, rank, dev) -> dict:
    """BASELINE config 4 (fibsem-mito-analysis): each rank owns a ``--em-z``-slice z-slab of a
    2048 x 2048 synthetic EM volume (256 slices per GPU = the 2048^3 volume at N=8), written as its own
    ``.npy`` and read back memory-mapped like the app's gang job reads a volume source
    (``em.volume.VolumeSource``).  Timed, max over ranks: slab read + H2D, percentiles (all-reduced),
    slice-wise 768/64 tiled 2-D U-Net inference (graph pass onto the HIP convs) with blending, the
    sharded touching-object split (remove small, closing, EDT, peaks, marker watershed; halo exchange
    over RCCL at N > 1), global instance statistics, and ``dist.gather`` of the int32 label volume
    onto rank 0 (reference: ``apps/fibsem-mito-analysis/analysis_deployment.py:108-176``, which is 2-D
    and CPU-side).  Stage timings are rank 0's."""
    import shutil
    import tempfile

    import numpy as np

    from bioengine_worker_amd.bioimageio.package import write_unet2d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.em.volume import VolumeSource, analyze_volume, gather_to_rank0
    from tools.em_volume_bench import synthetic_slab

    Z, YX = args.em_z, args.em_yx
    work = Path(tempfile.mkdtemp(prefix=f"be-em-bench-{rank}-", dir=os.environ.get("TMPDIR")))
    try:
        root = work / "mito-unet2d"
        write_unet2d_package(root, "mito-unet2d", in_channels=1, out_channels=1, features=(32, 64, 128, 256),
                             test_shape=(1, 1, 128, 128), torchscript=False)
        pipe = PredictionPipeline(root, device=dev)
        predict = lambda t: next(iter(pipe.predict_tensors(t).values()))  # noqa: E731
        z0 = rank * Z
        npy = work / "slab.npy"
        np.save(npy, synthetic_slab(z0, z0 + Z, YX, YX, dev).cpu().numpy())
        src = VolumeSource(str(npy))
        # the memory-mapped slab is read-only; torch only reads it (straight into the H2D copy)
        warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
        # 768^2 tiles (stride 704: 3 x 3 per 2048^2 slice, 5.3 M px of U-Net work) beat 512^2 (5 x 5,
        # 6.6 M px): 565 vs 520 M voxel/s on a 64 x 2048^2 slab, profiles/r06/em2d/sweep_s10.txt
        tile, ov = getattr(args, "em_tile", 768), getattr(args, "em_overlap", 64)
        # One untimed pass over the whole slab, like a training bench's warm-up steps: the first pass
        # at full size pays ~0.5 s of one-time costs (allocator growth for the multi-GB stage
        # buffers, the first large radix sort / nonzero) that a 4-slice warm-up does not cover
        # (sweep_s10.txt: stats 0.36 -> 0.02 s, peaks 0.10 -> 0.014 s, normalize 0.08 -> 0.002 s).
        warm = torch.from_numpy(src.read(0, Z)).to(dev)
        analyze_volume(warm, predict, tile, ov, args.em_tile_batch, split_touching=True, norm_range=(90.0, 210.0))
        del warm
        _barrier(world)
        t0 = time.perf_counter()
        slab = torch.from_numpy(src.read(0, Z)).to(dev)
        t_read = time.perf_counter()
        res = analyze_volume(slab, predict, tile, ov, args.em_tile_batch, group=None, z_offset=z0, timings=True,
                             split_touching=True)
        tg = time.perf_counter()
        full = gather_to_rank0(res["labels_slab_t"])
        torch.cuda.synchronize(dev)
        t_gather = time.perf_counter() - tg
        _barrier(world)
        dt = _max_over_ranks(time.perf_counter() - t0, world)
        vox = Z * world * YX * YX
        timings = dict(res["timings_s"])
        timings["read_h2d"] = round(t_read - t0, 4)
        timings["gather_rank0"] = round(t_gather, 4)
        out = {"em_volume_voxels_per_sec": round(vox / dt, 1),
               "em_volume_config": {"volume": [Z * world, YX, YX], "slab_per_gpu": [Z, YX, YX], "tile": tile,
                                    "overlap": ov, "tiles_per_call": args.em_tile_batch,
                                    "model": "BioImage.IO 2-D U-Net 32-64-128-256 (random init, graph pass: "
                                             "HIP convs, skip concatenation and max-pool read in the conv loaders)",
                                    "source": "memory-mapped .npy slab per rank", "split_touching": True,
                                    "gather": "rank0 (dist.gather of int32 labels)", "seconds": round(dt, 3),
                                    "n_instances": res["n_instances"],
                                    "rank0_volume": list(full.shape) if full is not None else None,
                                    "stage_timings_s_rank0": timings}}
        del slab, full, res
        return out
    finally:
        shutil.rmtree(work, ignore_errors=True)


def bench_em_volume3d(args, world, rank, dev) -> dict:
    """BASELINE config 4 as real 3-D tiled inference: each rank's z-slab through a
    BioImage.IO 3-D U-Net (16-32-64-128, Conv3d 3x3x3 + BN + ReLU on the one-launch implicit-GEMM
    kernel after the graph pass), 64 x 256 x 256 tiles with 8 / 16 voxels of overlap blended by the
    separable Gaussian window (be_blend_gather), then the same sharded post-processing and rank-0
    gather as the 2-D line.  Slab size per rank from --em3d-z / --em3d-yx (the 2048^3 volume at N = 8
    is --em3d-z 256 --em3d-yx 2048: same code, longer run)."""
    import shutil
    import tempfile

    import numpy as np

    from bioengine_worker_amd.bioimageio.package import write_unet3d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
    from bioengine_worker_amd.em.volume import VolumeSource, analyze_volume, gather_to_rank0
    from tools.em_volume_bench import synthetic_slab

    Z, YX = args.em3d_z, args.em3d_yx
    work = Path(tempfile.mkdtemp(prefix=f"be-em3d-bench-{rank}-", dir=os.environ.get("TMPDIR")))
    try:
        root = work / "mito-unet3d"
        write_unet3d_package(root, "mito-unet3d", in_channels=1, out_channels=1, features=(16, 32, 64, 128),
                             test_shape=(1, 1, 16, 32, 32))
        pipe = PredictionPipeline(root, device=dev)
        predict3d = lambda t: next(iter(pipe.predict_tensors(t).values()))  # noqa: E731
        z0 = rank * Z
        npy = work / "slab.npy"
        np.save(npy, synthetic_slab(z0, z0 + Z, YX, YX, dev).cpu().numpy())
        src = VolumeSource(str(npy))
        warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
        # 64 x 256^2 tiles, 4 per call: 350 vs 239 M voxel/s for the 32 x 128^2 tiles of round 5 on a
        # 64 x 2048^2 slab (profiles/r06/em3d/tile_sweep_s4_s5.txt: fewer, larger launches, and the
        # z overlap costs 8 of 64 slices instead of 8 of 32)
        kw = dict(tile=getattr(args, "em3d_tile", 256), overlap=16, batch=getattr(args, "em3d_batch", 4),
                  tile_z=getattr(args, "em3d_tile_z", 64), overlap_z=8, split_touching=True)
        warm = torch.from_numpy(src.read(0, Z)).to(dev)  # one untimed full-slab pass (see the 2-D line)
        analyze_volume(warm, None, predict3d=predict3d, norm_range=(90.0, 210.0), **kw)
        del warm
        _barrier(world)
        t0 = time.perf_counter()
        slab = torch.from_numpy(src.read(0, Z)).to(dev)
        t_read = time.perf_counter()
        res = analyze_volume(slab, None, predict3d=predict3d, group=None, z_offset=z0, timings=True, **kw)
        tg = time.perf_counter()
        full = gather_to_rank0(res["labels_slab_t"])
        torch.cuda.synchronize(dev)
        t_gather = time.perf_counter() - tg
        _barrier(world)
        dt = _max_over_ranks(time.perf_counter() - t0, world)
        timings = dict(res["timings_s"])
        timings["read_h2d"] = round(t_read - t0, 4)
        timings["gather_rank0"] = round(t_gather, 4)
        out = {"em_volume3d_voxels_per_sec": round(Z * world * YX * YX / dt, 1),
               "em_volume3d_config": {"volume": [Z * world, YX, YX], "slab_per_gpu": [Z, YX, YX],
                                      "tile": [kw["tile_z"], kw["tile"], kw["tile"]], "overlap": [8, 16, 16],
                                      "tiles_per_call": kw["batch"],
                                      "model": "BioImage.IO 3-D U-Net 16-32-64-128 (random init, graph pass: "
                                               "3x3x3 convs as z-tap launches of the 2-D MFMA kernel, skip "
                                               "concatenation read in the decoder conv's loader)",
                                      "split_touching": True, "gather": "rank0", "seconds": round(dt, 3),
                                      "n_instances": res["n_instances"], "stage_timings_s_rank0": timings}}
        del slab, full, res
        return out
    finally:
        shutil.rmtree(work, ignore_errors=True)


def bench_model_runner_cpu(reps: int = 10) -> dict:
    """BASELINE config 1 (model-runner plumbing on CPU): one BioImage.IO 2-D U-Net package, a single
    256x256 tile through the runtime's prediction pipeline on the CPU (pre-processing, padding,
    forward, post-processing) -- the path ``apps/model-runner/runtime_deployment.py`` serves; reference
    ``/root/reference/apps/model-runner/runtime_deployment.py:234-312``.  Median of ``reps`` calls."""
    import tempfile

    import numpy as np

    from bioengine_worker_amd.bioimageio.package import write_unet2d_package
    from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

    with tempfile.TemporaryDirectory(prefix="be-mr-bench-") as d:
        root = write_unet2d_package(Path(d) / "unet2d", "unet2d-cpu", in_channels=1, out_channels=2,
                                    test_shape=(1, 1, 256, 256), torchscript=False)
        pipe = PredictionPipeline(root, device=torch.device("cpu"))
        x = np.random.default_rng(0).random((1, 1, 256, 256), dtype=np.float32)
        pipe.predict(x)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            pipe.predict(x)
            ts.append((time.perf_counter() - t) * 1e3)
        ts.sort()
        return {"model_runner_cpu_infer_ms": round(ts[len(ts) // 2], 2),
                "model_runner_cpu_config": {"model": "BioImage.IO 2-D U-Net 32-64-128-256 (random init)",
                                            "input": [1, 1, 256, 256], "device": "cpu",
                                            "threads": torch.get_num_threads()}}


def bench_train_cpsam(args, world, rank, dev, batch: int, steps: int, force_dp: bool = False, zero: bool = False):
    """Cellpose-SAM (ViT-L/8, 256x256 crops) fine-tune steps -- the reference app's own training
    workload -- on the HIP CPSAM engine; with world > 1 data-parallel over RCCL (bucketed fp32
    gradients, all-reduces overlapped with the segmented-graph backward).  ``force_dp`` runs that
    data-parallel path on one GPU over a 1-rank group (its overhead vs the single-GPU graph).
    ``zero``: the ZeRO-1 optimizer (bucketed reduce-scatter, AdamW on the rank's chunk, all-gather;
    parallel/ddp.py ShardedAdamW) instead of all-reduce + full AdamW."""
    from bioengine_worker_amd.models.cpsam import CPSAM
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, build_trainer, synthetic_train_batch

    cfg = TrainConfig(batch_size=batch, bsize=256, lr=1e-5, weight_decay=1e-4, bucket_mb=64.0, comm_bf16=False,
                      force_dp_path=force_dp, zero_adamw=zero)
    trainer = build_trainer(cfg, device=dev, world_size=world, rank=rank, net=CPSAM().randomize_(0))
    data = synthetic_train_batch(batch, 256, device=dev, seed=rank)
    for _ in range(3):
        trainer.step(*data)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.step(*data)
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    del trainer
    torch.cuda.empty_cache()
    return batch * steps * world / dt, dt / steps * 1e3


def bench_cpsam_infer(dev, batch: int = 8, steps: int = 4, lat_n: int = 10) -> dict:
    """Cellpose-SAM inference -- the reference app's default ``infer`` model
    (apps/cellpose-finetuning/main.py:4966-5144, bf16 Transformer :126-127): 512x512x3 images through
    cellpose 4's 256-tile / 0.1-overlap path (9 tiles per image), the ViT-L/8 engine (HIP attention,
    rel-pos, LayerNorm; hipBLASLt linear layers after the A/B against the in-house GEMM, lin1's bias +
    GELU in hipBLASLt's GELU_BIAS epilogue)
    replayed from its HIP graph, taper blend, dynamics (niter 200), flow QC and fill holes.
    Random-init weights, synthetic images."""
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells
    from bioengine_worker_amd.models.cpsam import CPSAM

    runner = CellposeRunner(net=CPSAM().randomize_(0), device=dev)
    imgs = torch.from_numpy(synthetic_cells(batch, 512, 512, nchan=3, seed=0)).to(dev)
    p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15)
    for _ in range(2):
        runner.eval(imgs, p)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.eval(imgs, p)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    one = imgs[:1]
    for _ in range(2):
        runner.eval(one, p)
    lat = []
    for _ in range(lat_n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m, _, _ = runner.eval(one, p)
        m.cpu()
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    gemm = runner.engine.GEMM
    del runner
    torch.cuda.empty_cache()
    return {"cpsam_infer_imgs_per_s": round(batch * steps / dt, 2),
            "cpsam_infer_p50_ms_batch1": round(lat[len(lat) // 2], 2),
            "cpsam_infer_config": {"model": "Cellpose-SAM ViT-L/8 (dim 1024, 24 blocks), random init",
                                   "image": [512, 512, 3], "batch": batch, "tiles": "256 / 0.1 overlap (9 per image)",
                                   "gemm": {"mt": "in-house macro-tile MFMA (gemm_mt)",
                                            "ltgelu": "hipBLASLt; lin1 + bias + GELU (tanh approximation) in one "
                                                      "GEMM epilogue (exact-GELU path: BE_CPSAM_INFER_GEMM=lib)"}
                                           .get(gemm, "hipBLASLt + HIP bias/exact-GELU pass"),
                                   "graph": "one HIP graph per tile count", "masks": "dynamics niter 200, QC 0.4"}}


def bench_train_autograd(dev, arch: str, batch: int, steps: int = 6, warmup: int = 2, bf16: bool = False) -> float:
    """Reference-algorithm fine-tune step: the network as a plain torch module, PyTorch
    autograd, torch.optim.AdamW (lr 1e-5, wd 1e-4) and cellpose's ``_loss_fn_seg`` (flows MSE against
    5x targets / 2 + BCE-with-logits on cellprob) on the same 256x256 crops as the native lines, fp32
    like the reference's training (apps/cellpose-finetuning/main.py:1350-1358, 1483-1546) or under
    bf16 autocast.  Returns samples/s."""
    import torch.nn.functional as F

    from bioengine_worker_amd.models.cpnet import CPnet
    from bioengine_worker_amd.models.cpsam import CPSAM

    torch.manual_seed(0)
    if arch == "cpsam":
        net, nch = CPSAM().randomize_(0), 3
    else:
        net, nch = CPnet().randomize_(0), 2
    net = net.to(dev).float().train()
    opt = torch.optim.AdamW(net.parameters(), lr=1e-5, weight_decay=1e-4)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(batch, nch, 256, 256, generator=g).to(dev)
    lbl = torch.randn(batch, 3, 256, 256, generator=g).to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            y = net(x)[0]
        y = y.float()
        loss = F.mse_loss(y[:, :2], 5.0 * lbl[:, 1:]) / 2.0 + \
            F.binary_cross_entropy_with_logits(y[:, -1], (lbl[:, 0] > 0.5).float())
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del net, opt
    torch.cuda.empty_cache()
    return batch * steps / dt


def bench_train(args, world, rank, dev, norm="auto"):
    from bioengine_worker_amd.train.cellpose_train import TrainConfig, synthetic_train_batch, build_trainer

    cfg = TrainConfig(batch_size=args.train_batch, bsize=256, lr=1e-5, weight_decay=1e-4, norm=norm)
    trainer = build_trainer(cfg, device=dev, world_size=world, rank=rank)
    batch = synthetic_train_batch(args.train_batch, cfg.bsize, device=dev, seed=rank)
    for _ in range(max(2, args.warmup)):
        trainer.step(*batch)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        trainer.step(*batch)
    _barrier(world)
    dt = _max_over_ranks(time.perf_counter() - t0, world)
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="512x512 images per step per GPU")
    ap.add_argument("--train-batch", type=int, default=8, help="256x256 crops per step per GPU")
    ap.add_argument("--train-steps", type=int, default=30, help="timed steps of each fine-tune line (10 read +-10 %% apart across runs)")
    ap.add_argument("--chunks", type=int, default=1, help="micro-batches of the two-stream net/mask pipeline")
    ap.add_argument("--sequential", action="store_true", help="headline: one eval() per step, no cross-batch overlap")
    ap.add_argument("--no-extras", action="store_true", help="skip latency / train / reference-algorithm extras")
    ap.add_argument("--no-served", action="store_true", help="skip the served (full worker stack) measurement")
    ap.add_argument("--served-seconds", type=float, default=4.0, help="seconds per served concurrency level")
    ap.add_argument("--cpsam-batch", type=int, default=8, help="256x256 crops per step per GPU (Cellpose-SAM)")
    ap.add_argument("--em-z", type=int, default=256, help="z-slices per GPU of the EM volume line (2048^3 at N=8)")
    ap.add_argument("--em-yx", type=int, default=2048)
    ap.add_argument("--em-tile-batch", type=int, default=16, help="768^2 tiles per U-Net call (EM volume line)")
    ap.add_argument("--no-em", action="store_true", help="skip the EM volume line")
    ap.add_argument("--em3d-z", type=int, default=256, help="z-slices per GPU of the 3-D U-Net EM line (2048^3 at N=8)")
    ap.add_argument("--em3d-yx", type=int, default=2048)
    ap.add_argument("--trace", default=None, metavar="PATH",
                    help="after the timed steps, run one more traced step and write a Chrome trace (rank 0)")
    args = ap.parse_args()

    world, rank, local = _dist_setup(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from bioengine_worker_amd.ops import _native

    _native.hip()  # fail loudly if the kernels are missing

    _progress("headline", rank)
    dt, runner, imgs, p, extra = bench_infer(args, world, rank, dev)
    total_imgs = args.batch * args.steps * world
    value = total_imgs / dt
    ms_per_step = dt / args.steps * 1e3
    out = {
        "metric": "cellpose_cyto3_512x512_imgs_per_sec",
        "value": round(value, 2),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (512x512x2 uint16 blob images, random-init CPnet weights)",
        "config": {
            "model": "cellpose-cyto3 CPnet (nbase 2-32-64-128-256, style on, BN folded)",
            "global_batch": args.batch * world,
            "seq_len": None,
            "image": [512, 512, 2],
            "pipeline": "normalize99 + 224-tile/0.1-overlap + CPnet + taper blend + dynamics(niter=200) + flow QC(0.4) + fill holes(min 15)",
            "parallelism": f"dp{world} (replica per GPU)",
            "batches": ("one eval() per step" if (args.sequential or args.chunks > 1) else
                        "cross-batch two-stream pipeline: batch i+1's network overlaps batch i's mask "
                        "recovery (CellposeRunner.stream); sequential rate in imgs_per_sec_sequential_batches"),
        },
    }
    out.update(extra)
    if not args.no_extras:
        _progress("latency / reference algorithm / masks", rank)
        try:
            if rank == 0:
                p50, p95 = bench_latency(runner, imgs, p)
                out["p50_latency_ms_batch1"] = round(p50, 3)
                out["p95_latency_ms_batch1"] = round(p95, 3)
                ref_dt = bench_reference_algorithm(runner, imgs, p)
                out["reference_algorithm_imgs_per_sec_per_gpu"] = round(args.batch / ref_dt, 2)
                out["vs_reference_algorithm"] = round((value / world) / (args.batch / ref_dt), 3)
                mr_ms, mr_n = bench_mask_recovery(dev, args.batch)
                out["mask_recovery_ms_per_image_150cells"] = round(mr_ms, 3)
                out["mask_recovery_masks_per_image"] = mr_n
                cl, cl_n = bench_cell_like(runner, imgs, p)
                out["imgs_per_sec_cell_like"] = round(cl, 2)
                out["cell_like_masks_per_image"] = cl_n
        except Exception as e:  # extras must never take the headline down
            out["extras_error"] = f"latency/ref: {type(e).__name__}: {e}"
        if world == 1 and not args.no_served:
            _progress("served cellpose", rank)
            try:
                out.update(bench_served(args.served_seconds))
            except Exception as e:  # noqa: BLE001
                out["extras_error_served"] = f"{type(e).__name__}: {e}"
        if rank == 0:
            _progress("vit embed", rank)
            try:
                out["vit_embed_imgs_per_s"] = round(bench_vit_embed(dev), 1)  # per GPU, batch 64, fp8
                out["vit_embed_config"] = {"model": "DINOv2 ViT-B/14", "image": 224, "batch": 64,
                                           "gemm_dtype": "fp8 e4m3", "gemm": "HIP be_gemm_fp8 (block-scaled MFMA, MX-fp8 activations)", "baseline_img_s_A100_fp16": 500}
            except Exception as e:  # noqa: BLE001
                out["extras_error_vit"] = f"{type(e).__name__}: {e}"
        if world == 1 and not args.no_served:
            _progress("served search", rank)
            try:
                out.update(bench_served_search(args.served_seconds))
            except Exception as e:  # noqa: BLE001
                out["extras_error_served_search"] = f"{type(e).__name__}: {e}"
        _progress("cpnet fine-tune", rank)
        try:
            tdt = bench_train(args, world, rank, dev)
            out["finetune_samples_per_sec"] = round(args.train_batch * args.train_steps * world / tdt, 2)
            out["finetune_config"] = {"crop": 256, "batch_per_gpu": args.train_batch, "optimizer": "fused AdamW (HIP)",
                                      "norm": "group (DP default)" if world > 1 else "batch (cellpose cyto3)",
                                      "grad_allreduce": "RCCL bucketed, overlapped" if world > 1 else "none (1 GPU)"}
            if world == 1:  # the DP default (GroupNorm) on one GPU, for comparison with the BN line
                tdt = bench_train(args, world, rank, dev, norm="group")
                out["finetune_groupnorm_samples_per_sec"] = round(args.train_batch * args.train_steps / tdt, 2)
        except Exception as e:
            out["extras_error_train"] = f"{type(e).__name__}: {e}"
        if not args.no_em:
            _progress("em 2-d", rank)
            try:
                out.update(bench_em_volume(args, world, rank, dev))
            except Exception as e:  # noqa: BLE001
                out["extras_error_em"] = f"{type(e).__name__}: {e}"
            _progress("em 3-d", rank)
            try:
                out.update(bench_em_volume3d(args, world, rank, dev))
            except Exception as e:  # noqa: BLE001
                out["extras_error_em3d"] = f"{type(e).__name__}: {e}"
        if rank == 0:
            try:
                out.update(bench_model_runner_cpu())
            except Exception as e:  # noqa: BLE001
                out["extras_error_model_runner"] = f"{type(e).__name__}: {e}"
        _progress("cpsam fine-tune", rank)
        try:
            sps, ms = bench_train_cpsam(args, world, rank, dev, args.cpsam_batch, args.train_steps)
            out["finetune_cpsam_samples_per_sec"] = round(sps, 2)
            out["finetune_cpsam_config"] = {"model": "Cellpose-SAM ViT-L/8 (dim 1024, 24 blocks)", "crop": 256,
                                            "batch_per_gpu": args.cpsam_batch, "ms_per_step": round(ms, 3),
                                            "engine": "HIP fwd/bwd engine, HIP-graph step" if world == 1 else
                                            "HIP fwd/bwd engine, segmented HIP-graph step, RCCL bucketed fp32 all-reduce overlapped",
                                            "parallelism": f"dp{world}"}
            if world > 1:  # the ZeRO-1 optimizer on the same DP step
                _progress("cpsam fine-tune, zero-1", rank)
                try:
                    spz, msz = bench_train_cpsam(args, world, rank, dev, args.cpsam_batch, args.train_steps, zero=True)
                    out["finetune_cpsam_zero_samples_per_sec"] = round(spz, 2)
                    out["finetune_cpsam_zero_ms"] = round(msz, 3)
                except Exception as e:  # noqa: BLE001
                    out["extras_error_train_cpsam_zero"] = f"{type(e).__name__}: {e}"
            if world == 1:
                sps1, ms1 = bench_train_cpsam(args, world, rank, dev, 1, args.train_steps)
                out["finetune_cpsam_batch1_samples_per_sec"] = round(sps1, 2)  # the reference's batch size
                out["finetune_cpsam_ms_b1"] = round(ms1, 3)
                # the world > 1 step path (segmented graph + bucket all-reduces) forced on this GPU
                import socket

                with socket.socket() as so:
                    so.bind(("127.0.0.1", 0))
                    port = so.getsockname()[1]
                dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                        device_id=dev)
                try:
                    _, msd = bench_train_cpsam(args, world, rank, dev, 1, args.train_steps, force_dp=True)
                    out["finetune_cpsam_dp_path_ms_b1"] = round(msd, 3)
                    _, msz = bench_train_cpsam(args, world, rank, dev, 1, args.train_steps, force_dp=True, zero=True)
                    out["finetune_cpsam_zero_dp_path_ms_b1"] = round(msz, 3)
                finally:
                    dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001
            out["extras_error_train_cpsam"] = f"{type(e).__name__}: {e}"
        if rank == 0:
            _progress("cpsam inference", rank)
            try:
                out.update(bench_cpsam_infer(dev))
            except Exception as e:  # noqa: BLE001
                out["extras_error_cpsam_infer"] = f"{type(e).__name__}: {e}"
        if rank == 0:
            # reference-algorithm anchors of the two fine-tune lines (plain autograd + torch AdamW)
            try:
                out["finetune_autograd_samples_per_sec"] = round(
                    bench_train_autograd(dev, "cpnet", args.train_batch), 2)
                out["finetune_cpsam_autograd_samples_per_sec"] = round(
                    bench_train_autograd(dev, "cpsam", args.cpsam_batch, steps=4), 2)
                out["finetune_cpsam_autograd_bf16_samples_per_sec"] = round(
                    bench_train_autograd(dev, "cpsam", args.cpsam_batch, steps=4, bf16=True), 2)
                out["finetune_autograd_config"] = {
                    "what": "plain PyTorch autograd + torch.optim.AdamW + cellpose _loss_fn_seg, same crops "
                            "and batch as the native lines, no augmentation", "dtype": "fp32 (reference); "
                            "*_bf16: torch.autocast bf16"}
            except Exception as e:  # noqa: BLE001
                out["extras_error_train_autograd"] = f"{type(e).__name__}: {e}"
    if world > 1 and not args.no_extras and not args.no_served:
        _progress("served node", rank)
        out.update(bench_served_node(args, world, rank))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
