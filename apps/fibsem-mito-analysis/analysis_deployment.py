"""EM mitochondria analysis app.

API parity with the reference ``MitoAnalysisDeployment``
(apps/fibsem-mito-analysis/analysis_deployment.py:41-286): ``ping`` and ``analyze(image,
pixel_size_nm, tile_size, overlap)`` returning labels, per-instance properties (area_um2,
aspect_ratio, eccentricity, centroids), count, shape, model and timing — plus ``analyze_volume``
for 3-D stacks.

Where the reference is a CPU deployment that ships every 512x512 tile to the model-runner service
through S3 (3 concurrent round trips), this deployment owns a GPU and runs the tiles in batches
through the model-runner's in-process pipeline (fused MFMA convs), stitches with the HIP
gather-blend kernel and post-processes on the GPU; ``model_runner_service`` switches to the
reference's remote mode (any model-runner service on the hub).
"""
from __future__ import annotations

import asyncio
import base64
import io
import json
import os
import time
from datetime import datetime
from pathlib import Path

import numpy as np
from hypha_rpc.utils.schema import schema_method
from pydantic import Field
from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 2, "num_gpus": 1, "memory": 8 * 1024 ** 3},
                  max_ongoing_requests=4)
class MitoAnalysisDeployment:
    def __init__(self, model_id: str = "mito-unet2d", model_runner_service: str | None = None,
                 tile_batch: int = 8, features: list | None = None) -> None:
        self.start_time = time.time()
        self.model_id = model_id
        self.remote_service = model_runner_service
        self.tile_batch = tile_batch
        self.features = features or [32, 64, 128, 256]
        self._pipe = None
        self._remote = None

    async def async_init(self) -> None:
        import asyncio

        if self.remote_service:
            from hypha_rpc import connect_to_server

            server = await connect_to_server({"server_url": os.environ.get("HYPHA_SERVER_URL"),
                                              "token": os.environ.get("HYPHA_TOKEN")})
            self._remote = await server.get_service(self.remote_service)
            return
        await asyncio.to_thread(self._load_local)

    def _load_local(self) -> None:
        from bioengine_worker_amd.bioimageio.package import write_unet2d_package
        from bioengine_worker_amd.bioimageio.runner import PredictionPipeline
        from bioengine_worker_amd.bioimageio.zoo import list_local_models

        local = list_local_models().get(self.model_id)
        if local is not None:
            root = local["dir"]
        else:
            root = Path(os.environ.get("HOME", ".")) / "model_zoo" / self.model_id
            if not (root / "rdf.yaml").exists():
                write_unet2d_package(root, self.model_id, in_channels=1, out_channels=1, features=tuple(self.features),
                                     test_shape=(1, 1, 128, 128), torchscript=False)
        self._pipe = PredictionPipeline(root)

    async def test_deployment(self) -> None:
        r = await self.analyze(image=(np.random.rand(64, 64) * 255).astype(np.uint8).tolist())
        assert r["image_shape"] == [64, 64]

    async def check_health(self) -> None:
        if self._pipe is None and self._remote is None:
            raise RuntimeError("no inference backend")

    # ------------------------------------------------------------------ inference
    def _predict_local(self, tiles):
        out = self._pipe.predict_tensors(tiles)
        return next(iter(out.values()))

    async def _predict_remote(self, tiles):
        import torch

        res = []
        for t in tiles:
            r = await self._remote.infer(model_id=self.model_id, inputs=t.cpu().numpy())
            res.append(torch.from_numpy(np.asarray(next(iter(r.values())))).to(tiles.device))
        return torch.cat(res)

    async def _probability(self, img_norm, tile_size: int, overlap: int):
        import asyncio

        import torch

        from bioengine_worker_amd.em import mito

        H, W = img_norm.shape
        if self._remote is not None:
            # remote path: collect tiles, infer over RPC, blend on the device
            stride = tile_size - overlap
            ys, xs = list(range(0, H, stride)), list(range(0, W, stride))
            padded = torch.nn.functional.pad(img_norm[None, None], (0, max(0, xs[-1] + tile_size - W), 0,
                                                                    max(0, ys[-1] + tile_size - H)), mode="replicate")[0, 0]
            t = torch.stack([padded[y:y + tile_size, x:x + tile_size] for y in ys for x in xs])[:, None]
            probs = await self._predict_remote(t)
            return mito.infer_tiled(img_norm, lambda tt, it=iter(torch.split(probs, self.tile_batch)): next(it),
                                    tile_size, overlap, self.tile_batch)
        if H <= tile_size and W <= tile_size:
            return await asyncio.to_thread(lambda: self._predict_local(img_norm[None, None])[0])
        return await asyncio.to_thread(mito.infer_tiled, img_norm, self._predict_local, tile_size, overlap, self.tile_batch)

    # ------------------------------------------------------------------ API
    @schema_method
    async def ping(self) -> dict:
        """Service status."""
        return {"status": "ok", "model": self.model_id,
                "model_runner": self.remote_service or "in-process (MI355X fused pipeline)",
                "uptime_s": round(time.time() - self.start_time, 1), "timestamp": datetime.now().isoformat()}

    @schema_method
    async def analyze(self, image: list = Field(..., description="2D grayscale EM image (H x W nested list)."),
                      pixel_size_nm: float = Field(5.0, description="Pixel size in nm."),
                      tile_size: int = Field(512, description="Tile edge length for tiled inference."),
                      overlap: int = Field(64, description="Overlap between adjacent tiles.")) -> dict:
        """Segment mitochondria in a 2D EM image; labels + per-instance morphometrics."""
        import asyncio

        import torch

        from bioengine_worker_amd.em import mito

        t0 = time.time()
        arr = np.asarray(image, dtype=np.float32)
        if arr.ndim != 2:
            raise ValueError(f"Expected 2-D image, got shape {arr.shape}.")
        H, W = arr.shape
        dev = self._pipe.device if self._pipe is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        img = mito.normalize_percentile(torch.from_numpy(arr).to(dev))
        prob = await self._probability(img, tile_size, overlap)
        prob = prob[0] if prob.dim() == 3 else prob
        if dev.type == "cuda":
            labels = await asyncio.to_thread(mito.prob_to_instances, prob)
        else:  # CPU deployments: scipy oracle of the same pipeline
            labels = await asyncio.to_thread(mito.prob_to_instances_cpu, prob.cpu().numpy())
        props = await asyncio.to_thread(mito.region_properties, labels, pixel_size_nm, dev)
        return {"labels": labels.tolist(), "properties": props, "n_mitochondria": int(labels.max()),
                "image_shape": [H, W], "pixel_size_nm": pixel_size_nm, "model": self.model_id,
                "processing_time_s": round(time.time() - t0, 2)}

    def _data_root(self) -> Path:
        return Path(os.environ.get("BIOENGINE_EM_DATA_ROOT") or Path(os.environ.get("HOME", ".")) / "em_data").resolve()

    def _volume_spec(self, volume_npy_b64, volume_path, dataset_id, dataset_file, array, work: Path) -> dict:
        """Where the ranks read the volume from (each reads only its z-slab): an uploaded ``.npy``
        (written once to local disk, memory-mapped by the ranks), a ``.npy`` / ``.zarr`` path under
        ``BIOENGINE_EM_DATA_ROOT``, or a zarr array of a BioEngine dataset (HTTP range reads,
        reference ``bioengine/datasets/http_zarr_store.py``)."""
        given = [x is not None for x in (volume_npy_b64, volume_path, dataset_id)]
        if sum(given) != 1:
            raise ValueError("give exactly one of volume_npy_b64, volume_path, dataset_id")
        if volume_npy_b64 is not None:
            vpath = work / "volume.npy"
            vpath.write_bytes(base64.b64decode(volume_npy_b64))
            return {"kind": "npy", "path": str(vpath)}
        if volume_path is not None:
            root = self._data_root()
            p = (root / volume_path).resolve() if not Path(volume_path).is_absolute() else Path(volume_path).resolve()
            if p != root and root not in p.parents:  # paths are caller input: never outside the data root
                raise PermissionError(f"volume_path must lie under {root}")
            if not p.exists():
                raise FileNotFoundError(str(p))
            kind = "zarr" if p.is_dir() else "npy"
            return {"kind": kind, "path": str(p), "array": array or ""}
        ds = getattr(self, "bioengine_datasets", None)
        if ds is None or not getattr(ds, "data_server_url", None):
            raise RuntimeError("no BioEngine datasets server is configured for this worker")
        f = str(dataset_file or "")
        if ".zarr" not in f:
            raise ValueError("dataset_file must name a .zarr array")
        rootf = f.split(".zarr")[0] + ".zarr"
        inner = (f.split(".zarr", 1)[1].strip("/") or array or "")
        return {"kind": "dataset", "url": f"{ds.data_server_url}/data/{dataset_id}/{rootf}", "array": inner,
                "token": getattr(ds, "token", None)}

    def _model3d_root(self, model_id_3d: str) -> str:
        """Directory of an installed 3-D model.  Only ids already present in the local zoo resolve;
        the id is caller input, so it is never turned into a path of its own, and a missing model is
        an error (no placeholder weights are ever written under the caller's id)."""
        from bioengine_worker_amd.bioimageio.zoo import list_local_models

        local = list_local_models().get(str(model_id_3d))
        if local is None:
            raise FileNotFoundError(f"no installed 3-D model '{model_id_3d}' in the local model zoo; "
                                    "install one (model-runner) or use inference='slice2d'")
        root = Path(local["dir"]).resolve()
        if not (root / "rdf.yaml").exists():
            raise FileNotFoundError(f"model '{model_id_3d}' has no rdf.yaml")
        return str(root)

    @schema_method
    async def analyze_volume(self, volume_npy_b64: str | None = Field(None, description="3-D stack as base64 .npy bytes (Z,Y,X)."),
                             volume_path: str | None = Field(None, description="A .npy file or .zarr directory under "
                                                                               "BIOENGINE_EM_DATA_ROOT (no upload: every "
                                                                               "GPU reads only its z-slab)."),
                             dataset_id: str | None = Field(None, description="BioEngine dataset holding the volume."),
                             dataset_file: str | None = Field(None, description="Zarr array in that dataset, e.g. 'em.zarr/raw'."),
                             array: str | None = Field(None, description="Array path inside a zarr group."),
                             pixel_size_nm: float = Field(5.0, description="In-plane pixel size in nm."),
                             tile_size: int = Field(512, description="Tile edge length."),
                             overlap: int = Field(64, description="Tile overlap."),
                             n_gpus: int = Field(1, description="Shard z-slabs over this many GPUs (gang job, RCCL)."),
                             gather: str = Field("rank0", description="n_gpus > 1: 'rank0' stitches the label volume on "
                                                                      "one GPU, 'sharded' keeps per-slab files, "
                                                                      "'none' returns statistics only."),
                             return_labels: bool = Field(False, description="Include the label volume (base64 .npy)."),
                             threshold: float = Field(0.5, description="Foreground probability threshold."),
                             input_is_probability: bool = Field(False, description="The volume already is a foreground "
                                                                                   "probability map (skip the model)."),
                             split_touching: bool = Field(False, description="Separate touching mitochondria: the "
                                                                             "reference post-processing (remove small, "
                                                                             "closing, EDT, peaks, watershed) in 3-D, "
                                                                             "sharded across the GPUs."),
                             closing_radius: int = Field(4, description="Closing disk radius (split_touching)."),
                             min_distance: int = Field(8, description="Peak min distance (split_touching)."),
                             min_voxels: int = Field(300, description="Smallest instance kept (voxels)."),
                             inference: str = Field("slice2d", description="'slice2d' (2-D tiles per slice) or "
                                                                           "'tiled3d' (3-D tiles, 3-D U-Net, z-overlap blend)."),
                             model_id_3d: str = Field("mito-unet3d", description="3-D model for inference='tiled3d'."),
                             tile_z: int = Field(32, description="3-D tile depth."),
                             overlap_z: int = Field(8, description="3-D tile z-overlap."),
                             ) -> dict:
        """3-D mitochondria instances with per-instance volume.  With ``n_gpus > 1`` the z-slabs run
        as one rank per GPU (each reads only its slab) with globally consistent labels."""
        import shutil
        import tempfile

        import torch

        from bioengine_worker_amd.em import volume as vol

        if inference not in ("slice2d", "tiled3d"):
            raise ValueError("inference must be 'slice2d' or 'tiled3d'")
        if self._pipe is None and not input_is_probability:
            raise RuntimeError("volume analysis needs the in-process pipeline (no model_runner_service)")
        work = Path(tempfile.mkdtemp(prefix="em-vol-", dir=os.environ.get("TMPDIR")))
        spec = await asyncio.to_thread(self._volume_spec, volume_npy_b64, volume_path, dataset_id, dataset_file, array, work)
        model3d = None
        if inference == "tiled3d" and not input_is_probability:
            model3d = await asyncio.to_thread(self._model3d_root, model_id_3d)
        t0 = time.time()
        kw = {"volume": spec, "model_root": None if (input_is_probability or model3d) else str(self._pipe.root),
              "model3d_root": model3d, "tile": tile_size, "overlap": overlap, "batch": self.tile_batch,
              "threshold": float(threshold), "min_voxels": int(min_voxels), "split_touching": bool(split_touching),
              "closing_radius": int(closing_radius), "min_distance": int(min_distance), "tile_z": int(tile_z),
              "overlap_z": int(overlap_z)}
        opath = work / "labels.npy"
        try:
            if int(n_gpus or 1) > 1:
                from bioengine_worker_amd.serve.gang import run_gang

                res = await run_gang("bioengine_worker_amd.em.volume:gang_analyze_volume",
                                     dict(kw, out_path=str(opath), gather=gather),
                                     world_size=int(n_gpus), gpus_per_rank=1, name=f"em-{work.name[-8:]}")
                out = dict(res[0])
                out.update(ranks=[{k: r[k] for k in ("rank", "z_range", "timings_s", "gather_s", "total_s")} for r in res],
                           n_gpus=int(n_gpus), gather=gather, processing_time_s=round(time.time() - t0, 2))
                if return_labels and gather == "rank0":
                    out["labels_npy_b64"] = base64.b64encode(opath.read_bytes()).decode()
                elif gather == "sharded":
                    out["label_shards"] = json.loads(Path(f"{opath}.manifest.json").read_text())
            else:
                def run_local():
                    dev = self._pipe.device if self._pipe is not None else torch.device("cpu")
                    src = vol.VolumeSource(spec)
                    v = torch.from_numpy(src.read(0, src.shape[0]).astype(np.float32)).to(dev)
                    p1, p99 = src.percentiles(dev)
                    predict3d = None
                    if model3d:
                        from bioengine_worker_amd.bioimageio.runner import PredictionPipeline

                        p3 = PredictionPipeline(model3d, device=dev)
                        predict3d = lambda t: next(iter(p3.predict_tensors(t).values()))
                    predict = vol.probability_identity if input_is_probability else self._predict_local
                    r = vol.analyze_volume(v, predict, tile_size, overlap, self.tile_batch, threshold=float(threshold),
                                           min_voxels=int(min_voxels), norm_range=(float(p1), float(p99)),
                                           split_touching=bool(split_touching), closing_radius=int(closing_radius),
                                           min_distance=int(min_distance), predict3d=predict3d, tile_z=int(tile_z),
                                           overlap_z=int(overlap_z))
                    labels = r.pop("labels_slab_t")
                    if return_labels:
                        b = io.BytesIO()
                        np.save(b, labels.cpu().numpy())
                        r["labels_npy_b64"] = base64.b64encode(b.getvalue()).decode()
                    return r

                out = await asyncio.to_thread(run_local)
                out.update(split_touching=bool(split_touching), inference=inference,
                           processing_time_s=round(time.time() - t0, 2))
        finally:
            if gather != "sharded" or int(n_gpus or 1) <= 1:
                shutil.rmtree(work, ignore_errors=True)
        out["pixel_size_nm"] = pixel_size_nm
        out["model"] = model_id_3d if model3d else self.model_id
        return out
