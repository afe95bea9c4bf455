"""Training-data discovery for the cellpose-finetuning app: artifact listing, glob / folder pairing of
images with annotations, metadata-JSON pairing, cached downloads and label decoding.

Behaviour follows the reference app's data layer (``apps/cellpose-finetuning/main.py:2321-3140``:
``list_matching_artifact_paths``, ``match_image_annotation_pairs``,
``make_training_pairs_from_metadata``, ``download_pairs_from_artifact``, ``create_dataset_split``;
label decoding ``:337-414``) and is pinned by the reference's own offline tests
(``tests/apps/cellpose/test_metadata_and_glob.py``), which run against this module through the app.

The artifact handle only needs two coroutines, matching hypha's ``AsyncHyphaArtifact``:
``ls(folder) -> [{"path"|"name", "type"}]`` and ``get(remote_paths, local_paths, on_error)``.
:class:`HubArtifact` provides them on top of any artifact-manager service (ours or Hypha's).
"""
from __future__ import annotations

import fnmatch
import io
import json
import logging
import os
import posixpath
import re
from pathlib import Path
from typing import Any

import numpy as np

log = logging.getLogger("bioengine.cellpose.datasets")

IMAGE_SUFFIXES = (".ome.tiff", ".ome.tif", ".tiff", ".tif", ".png", ".jpg", ".jpeg", ".npy")
ANNOTATION_MARKERS = ("_mask", "-mask", "_label", "-label", "_annotation", "-annotation")
PAIR_TOKENS = ("image", "mask", "annotation", "label", "input", "target")
RECORD_LISTS = ("records", "items", "samples", "entries", "data")
IMAGE_KEYS = ("image", "image_path", "imagepath", "imagePath", "image_relpath", "imageRelPath", "image_file",
              "imageFile", "raw", "raw_image", "rawImage", "input", "input_path", "inputPath", "input_image",
              "inputImage", "source", "source_path", "sourcePath", "img")
ANNOTATION_KEYS = ("annotation", "annotation_path", "annotationPath", "annotation_relpath", "annotationRelPath",
                   "annotation_file", "annotationFile", "mask", "mask_path", "maskPath", "mask_relpath",
                   "maskRelPath", "mask_file", "maskFile", "label", "label_path", "labelPath", "label_file",
                   "labelFile", "labels", "target", "target_path", "targetPath", "gt", "ground_truth",
                   "groundTruth")
TEST_SPLITS = {"test", "val", "validation"}


class MetadataPairError(ValueError):
    """Metadata JSON files exist but none of their records names an (image, annotation) pair."""


# ------------------------------------------------------------------ paths / patterns
def rel(p: str | Path) -> str:
    """Artifact-relative POSIX path (no leading slash, forward slashes)."""
    return str(p).replace("\\", "/").lstrip("/")


def safe_rel(p: str | Path) -> str:
    """:func:`rel` normalised, refusing any path that climbs out of its root (``..``).  Paths in a
    user's metadata JSON are untrusted: without this a record could point training at another
    session's files or make a download land outside the cache directory."""
    r = posixpath.normpath(rel(p)) if rel(p) else ""
    if r in ("", "."):
        raise ValueError(f"empty artifact path: {p!r}")
    if r == ".." or r.startswith("../") or "\x00" in r:
        raise ValueError(f"artifact path escapes its root: {p!r}")
    return r


def local_path(root: Path, remote: str | Path) -> Path:
    """Local cache location of an artifact file; must stay under ``root`` (symlinks included)."""
    root = Path(root)
    lp = root / safe_rel(remote)
    base = root.resolve()
    res = lp.resolve()
    if res != base and base not in res.parents:
        raise ValueError(f"artifact path escapes the cache directory: {remote!r}")
    return lp


def _glob_regex(pattern: str) -> re.Pattern:
    parts = [re.escape(x) for x in rel(pattern).split("*")]
    return re.compile("^" + "(.+?)".join(parts) + "$")


def pattern_captures(path: str, pattern: str) -> tuple[str, ...] | None:
    """The strings the ``*`` wildcards of ``pattern`` matched in ``path`` (None: no match).  A
    wildcard may span directory separators, like a shell ``**`` segment."""
    if "*" not in pattern:
        return () if rel(path) == rel(pattern) else None
    m = _glob_regex(pattern).match(rel(path))
    return tuple(m.groups()) if m else None


def _strip_suffix(name: str) -> str:
    low = name.lower()
    for suf in IMAGE_SUFFIXES:
        if low.endswith(suf):
            return name[: -len(suf)]
    return Path(name).stem


def _image_key(path: str) -> str:
    return _strip_suffix(Path(path).name).lower()


def _annotation_key(path: str) -> str:
    key = _strip_suffix(Path(path).name).lower()
    for marker in ANNOTATION_MARKERS:
        if key.endswith(marker):
            return key[: -len(marker)]
    return key


def match_image_annotation_pairs(image_files: list[str], annotation_files: list[str], image_pattern: str,
                                 annotation_pattern: str) -> list[tuple[str, str]]:
    """Pair images with annotations whose wildcard captures agree (``images/*/*.tif`` with
    ``annotations/*/*_mask.ome.tif``).  If no capture pairs exist (mixed naming conventions such as
    ``*.tif`` vs ``*_mask.ome.tif``), fall back to base-name keys with image suffixes and mask markers
    (``_mask``, ``-label``, ...) removed."""
    by_capture: dict[tuple[str, ...], str] = {}
    for a in annotation_files:
        cap = pattern_captures(a, annotation_pattern)
        if cap:
            by_capture[cap] = a
    pairs = []
    for im in image_files:
        cap = pattern_captures(im, image_pattern)
        if cap and cap in by_capture:
            pairs.append((im, by_capture[cap]))
    if pairs:
        return pairs
    by_key: dict[str, str] = {}
    for a in annotation_files:
        by_key.setdefault(_annotation_key(a), a)
    return [(im, by_key[_image_key(im)]) for im in image_files if _image_key(im) in by_key]


# ------------------------------------------------------------------ listing
def _entry(e: Any) -> tuple[str, bool]:
    if isinstance(e, dict):
        p = str(e.get("path") or e.get("name") or "")
        t = str(e.get("type") or "").lower()
    else:
        p, t = str(e), ""
    p = rel(p)
    return p, (p.endswith("/") or t in ("folder", "directory", "dir"))


async def list_artifact_files(artifact, folder: str) -> list[str]:
    """Base names of the entries directly under ``folder``."""
    folder = rel(folder)
    folder = folder if folder.endswith("/") or not folder else folder + "/"
    out = []
    for e in await artifact.ls(folder):
        p, _ = _entry(e)
        name = Path(p).name
        if name and name != ".":
            out.append(name)
    return out


async def list_artifact_files_recursive(artifact, folder: str) -> list[str]:
    """Every file path (artifact-relative) under ``folder``, breadth first, sorted."""
    root = rel(folder)
    if root and not root.endswith("/"):
        root += "/"
    todo, seen, files = [root], set(), set()
    while todo:
        cur = todo.pop(0)
        if cur in seen:
            continue
        seen.add(cur)
        for e in await artifact.ls(cur):
            p, is_dir = _entry(e)
            if cur and p and not p.startswith(cur):
                p = rel(cur + p)
            if is_dir:
                todo.append(p if p.endswith("/") else p + "/")
            elif p:
                files.add(p)
    return sorted(files)


def _glob_root(pattern: str) -> str:
    p = rel(pattern)
    star = p.find("*")
    if star < 0:
        return p if p.endswith("/") else str(Path(p).parent) + "/"
    cut = p.rfind("/", 0, star)
    return "" if cut < 0 else p[: cut + 1]


async def list_matching_artifact_paths(artifact, path_pattern: str) -> list[str]:
    """Files matching a folder (``images/`` or ``images`` -- a trailing slash is optional) or a glob
    (``images/*/*.tif``; the listing is recursive below the part before the first wildcard)."""
    pat = rel(path_pattern)
    if pat.endswith("/"):
        return [rel(pat + n) for n in await list_artifact_files(artifact, pat)]
    if "*" not in pat:
        try:
            entries = await artifact.ls(pat)
        except Exception:  # noqa: BLE001  (not a folder: a single file path)
            entries = None
        if isinstance(entries, list) and entries:
            return [rel(pat + "/" + n) for n in await list_artifact_files(artifact, pat)]
        return [pat]
    cands = await list_artifact_files_recursive(artifact, _glob_root(pat))
    return sorted({c for c in cands if fnmatch.fnmatch(c, pat)})


# ------------------------------------------------------------------ downloads
def _missing(paths: list[str], root: Path) -> tuple[list[str], list[str]]:
    rem, loc = [], []
    for p in paths:
        lp = local_path(root, p)
        if not lp.exists() or lp.stat().st_size <= 0:
            lp.parent.mkdir(parents=True, exist_ok=True)
            rem.append(rel(p))
            loc.append(str(lp))
    return rem, loc


async def download_pairs_from_artifact(artifact, out_dir: Path, image_paths: list, annotation_paths: list,
                                       timeout_s: float = 600.0) -> list[dict]:
    """Fetch the files not yet cached under ``out_dir`` and return local ``{image, annotation}`` pairs."""
    import asyncio

    out_dir = Path(out_dir)
    rem, loc = _missing([str(p) for p in [*image_paths, *annotation_paths]], out_dir)
    if rem:
        log.info("downloading %d dataset files", len(rem))
        try:
            await asyncio.wait_for(artifact.get(rem, loc, on_error="ignore"), timeout=timeout_s)
        except asyncio.TimeoutError:
            raise RuntimeError(f"Download of {len(rem)} files timed out after {timeout_s:.0f} s") from None
    imgs = [local_path(out_dir, p) for p in image_paths]
    anns = [local_path(out_dir, p) for p in annotation_paths]
    gone = [str(p) for p in [*imgs, *anns] if not p.exists() or p.stat().st_size <= 0]
    if gone:
        raise RuntimeError(f"{len(gone)} dataset files missing after download (e.g. {', '.join(gone[:5])}); "
                           "check the paths / metadata against the artifact contents")
    return [{"image": i, "annotation": a} for i, a in zip(imgs, anns)]


# ------------------------------------------------------------------ metadata JSON
def _pair_records(payload: Any) -> list[dict]:
    """Every dict in the JSON tree whose keys look like an (image, annotation) record."""
    found, stack, seen = [], [payload], set()
    while stack:
        cur = stack.pop()
        if id(cur) in seen:
            continue
        seen.add(id(cur))
        if isinstance(cur, list):
            stack.extend(reversed(cur))
        elif isinstance(cur, dict):
            keys = [str(k).lower() for k in cur]
            if any(tok in k for k in keys for tok in PAIR_TOKENS):
                found.append(cur)
            stack.extend(v for v in cur.values() if isinstance(v, (dict, list)))
    if found:
        return found
    if isinstance(payload, list):
        return [x for x in payload if isinstance(x, dict)]
    if isinstance(payload, dict):
        for k in RECORD_LISTS:
            if isinstance(payload.get(k), list):
                return [x for x in payload[k] if isinstance(x, dict)]
        return [payload]
    return []


def _record_path(value: Any, parent: Path) -> Path | None:
    if isinstance(value, dict):
        for k in ("path", "file", "uri", "name"):
            if k in value:
                return _record_path(value[k], parent)
        return None
    if not isinstance(value, str) or not value.strip():
        return None
    v = value.strip().replace("\\", "/")
    if v.startswith(("http://", "https://")):
        return None
    try:
        if v.startswith("/"):
            return Path(safe_rel(v))
        if "/" in v and not v.startswith("./"):
            return Path(safe_rel(v))  # artifact-relative
        return Path(safe_rel(parent / v))  # relative to the metadata file's folder
    except ValueError:
        return None  # a path that leaves the artifact is not a usable record


def _record_pair(rec: dict, parent: Path) -> dict | None:
    def first(keys):
        for k in keys:
            p = _record_path(rec.get(k), parent)
            if p is not None:
                return p
        return None

    img, ann = first(IMAGE_KEYS), first(ANNOTATION_KEYS)
    return None if img is None or ann is None else {"image": img, "annotation": ann}


def _is_test(rec: dict) -> bool:
    split = rec.get("split") or rec.get("dataset_split") or rec.get("subset") or rec.get("partition") or "train"
    return str(split).lower() in TEST_SPLITS


async def make_training_pairs_from_metadata(artifact, metadata_dir: str, save_path: Path,
                                            n_samples: int | None) -> tuple[list[dict], list[dict]]:
    """(train_pairs, test_pairs) from every ``*.json`` under ``metadata_dir`` (records may be nested
    under payload/items/...; keys in snake or camel case; paths absolute, artifact-relative or
    relative to the JSON file; ``split``/``subset`` = test|val|validation marks test records)."""
    root = rel(metadata_dir)
    if root and not root.endswith("/"):
        root += "/"
    files = [p for p in await list_artifact_files_recursive(artifact, root) if p.lower().endswith(".json")]
    if not files:
        raise ValueError(f"No metadata JSON files found under '{metadata_dir}'")
    save_path = Path(save_path)
    rem, loc = _missing(files, save_path)
    if rem:
        await artifact.get(rem, loc, on_error="ignore")
    train, test = [], []
    for f in files:
        lp = local_path(save_path, f)
        if not lp.exists():
            continue
        payload = json.loads(lp.read_text(encoding="utf-8"))
        for rec in _pair_records(payload):
            pr = _record_pair(rec, Path(f).parent)
            if pr is not None:
                (test if _is_test(rec) else train).append(pr)
    if not train:
        raise MetadataPairError("No training pairs found in the metadata JSON files (expected keys such as "
                                "image_path / mask_path, camelCase accepted)")
    if n_samples is not None and n_samples < len(train):
        keep = np.random.default_rng().permutation(len(train))[:n_samples]
        train = [train[i] for i in keep]
    train_pairs = await download_pairs_from_artifact(artifact, save_path, [p["image"] for p in train],
                                                     [p["annotation"] for p in train])
    test_pairs = []
    if test:
        test_pairs = await download_pairs_from_artifact(artifact, save_path, [p["image"] for p in test],
                                                        [p["annotation"] for p in test])
    return train_pairs, test_pairs


async def make_training_pairs(artifact, params: dict, save_path: Path) -> tuple[list[dict], list[dict]]:
    """Training/test pairs for a session's parameters (``metadata_dir`` first, then the
    ``train_images`` / ``train_annotations`` patterns), downloaded into ``save_path``."""
    ti, ta = params.get("train_images"), params.get("train_annotations")
    if params.get("metadata_dir"):
        try:
            return await make_training_pairs_from_metadata(artifact, params["metadata_dir"], save_path,
                                                           params.get("n_samples"))
        except MetadataPairError as e:
            if not (ti and ta):
                raise
            log.warning("metadata gave no pairs (%s); using train_images/train_annotations", e)
    if not (ti and ta):
        raise ValueError("Either metadata_dir, or both train_images and train_annotations must be provided.")

    async def pairs_for(ip, ap, n=None):
        ims = await list_matching_artifact_paths(artifact, ip)
        ans = await list_matching_artifact_paths(artifact, ap)
        matched = match_image_annotation_pairs(ims, ans, ip, ap)
        if n is not None and n < len(matched):
            keep = np.random.default_rng().permutation(len(matched))[:n]
            matched = [matched[i] for i in keep]
        return await download_pairs_from_artifact(artifact, save_path, [a for a, _ in matched],
                                                  [b for _, b in matched])

    train = await pairs_for(ti, ta, params.get("n_samples"))
    test = []
    if params.get("test_images") and params.get("test_annotations"):
        test = await pairs_for(params["test_images"], params["test_annotations"])
    return train, test


# ------------------------------------------------------------------ image / label IO
def read_image(path: str | Path) -> np.ndarray:
    """npy, or any PIL-readable image (multi-page TIFF -> stacked frames)."""
    p = Path(path)
    if p.suffix.lower() == ".npy":
        return np.load(p, allow_pickle=False)
    return decode_image(p.read_bytes())


def decode_image(data: bytes, name: str = "") -> np.ndarray:
    if name.endswith(".npy") or data[:6] == b"\x93NUMPY":
        return np.load(io.BytesIO(data), allow_pickle=False)
    from PIL import Image

    img = Image.open(io.BytesIO(data))
    frames = []
    i = 0
    while True:
        try:
            img.seek(i)
        except EOFError:
            break
        frames.append(np.array(img))
        i += 1
    return frames[0] if len(frames) == 1 else np.stack(frames)


def decode_labels(arr: np.ndarray) -> np.ndarray:
    """Instance labels from any annotation encoding: palette/grey images as they are, RGB(A) images
    either as 16-bit ids split over R (high) and G (low) with B == 0 (colab annotation export) or as
    the R channel (reference ``_load_label_array``, main.py:392-414)."""
    a = np.asarray(arr)
    if a.ndim == 3 and a.shape[-1] in (3, 4):
        r, g, b = a[..., 0].astype(np.uint32), a[..., 1].astype(np.uint32), a[..., 2]
        a = (r << 8) | g if not np.any(b) else a[..., 0]
    return np.asarray(a).astype(np.int32)


def read_labels(path: str | Path) -> np.ndarray:
    return decode_labels(read_image(path))


def has_foreground(path: str | Path) -> bool:
    try:
        lab = read_labels(path)
    except Exception as e:  # noqa: BLE001
        log.warning("skipping unreadable annotation %s: %s", path, e)
        return False
    if lab.ndim != 2:
        log.warning("skipping non-2D annotation %s (shape %s)", path, lab.shape)
        return False
    return bool((lab > 0).any())


def create_dataset_split(train_pairs: list[dict], test_pairs: list[dict]) -> dict:
    """Drop pairs whose annotation has no foreground (reference ``create_dataset_split``)."""
    tr = [p for p in train_pairs if has_foreground(p["annotation"])]
    te = [p for p in test_pairs if has_foreground(p["annotation"])]
    if not tr:
        raise ValueError("No training pairs found. At least one training sample is required.")
    return {"train_files": [p["image"] for p in tr], "train_labels_files": [p["annotation"] for p in tr],
            "test_files": [p["image"] for p in te] or None, "test_labels_files": [p["annotation"] for p in te] or None}


# ------------------------------------------------------------------ artifact handle
class HubArtifact:
    """``ls`` / ``get`` over an artifact-manager service (our hub or Hypha)."""

    def __init__(self, artifact_manager, artifact_id: str, timeout_s: float = 120.0):
        self.am, self.aid, self.timeout_s = artifact_manager, artifact_id, timeout_s

    async def ls(self, folder: str):
        d = rel(folder).rstrip("/")
        entries = await self.am.list_files(self.aid, dir_path=d or None)
        base = d + "/" if d else ""
        out = []
        for e in entries:
            name = e.get("name") if isinstance(e, dict) else getattr(e, "name", str(e))
            typ = e.get("type") if isinstance(e, dict) else getattr(e, "type", "file")
            out.append({"path": base + str(name) + ("/" if typ == "directory" else ""), "type": typ})
        return out

    async def get(self, remote_paths: list[str], local_paths: list[str], on_error: str = "raise"):
        import httpx

        async with httpx.AsyncClient(timeout=self.timeout_s) as c:
            for rp, lp in zip(remote_paths, local_paths):
                try:
                    url = await self.am.get_file(self.aid, file_path=rel(rp))
                    r = await c.get(url)
                    r.raise_for_status()
                    Path(lp).parent.mkdir(parents=True, exist_ok=True)
                    tmp = str(lp) + ".part"
                    with open(tmp, "wb") as f:
                        f.write(r.content)
                    os.replace(tmp, lp)
                except Exception:  # noqa: BLE001
                    if on_error != "ignore":
                        raise
