"""Cellpose model identities for the apps: built-in models, fine-tuned session checkpoints, weights.

* Built-ins (reference ``PretrainedModel``, ``apps/cellpose-finetuning/main.py:434-446``):
  ``cpsam`` -- Cellpose-SAM (cellpose 4, ViT-L/8) -- the reference's only and default model, and
  ``cyto3`` -- the cellpose 3 CPnet U-Net (the model-runner's cellpose pin).
* Offline there are no pretrained checkpoints.  ``BIOENGINE_CPSAM_WEIGHTS`` /
  ``BIOENGINE_CYTO3_WEIGHTS`` point at a local state dict (loaded with ``weights_only=True``);
  without one the built-in is randomly initialised and :func:`build_net` reports
  ``weights="random"`` so callers can surface it.
* Session checkpoints are ``{"arch", "arch_kwargs", "state_dict"}`` dicts (tensors + plain types
  only, so ``weights_only=True`` loads them).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

BUILTIN_MODELS = {
    "cpsam": "Cellpose-SAM 4.0 model (transformer-based, channel-order invariant).",
    "cyto3": "Cellpose 3 cyto3 CPnet U-Net (residual conv blocks, style vector).",
}
WEIGHTS_ENV = {"cpsam": "BIOENGINE_CPSAM_WEIGHTS", "cyto3": "BIOENGINE_CYTO3_WEIGHTS"}
# Cellpose-SAM encoder sizes: vit_l is cellpose 4's; the small ones keep CPU tests and demos cheap
CPSAM_ARCHS = {"vit_l": dict(dim=1024, depth=24, heads=16), "vit_b": dict(dim=768, depth=12, heads=12),
               "tiny": dict(dim=128, depth=2, heads=2)}


def new_net(arch: str, arch_kwargs: dict | None = None):
    kw = dict(arch_kwargs or {})
    if arch == "cpsam":
        from ..models.cpsam import CPSAM

        return CPSAM(**kw)
    if arch == "cpnet":
        from ..models.cpnet import CPnet

        return CPnet(**kw)
    raise ValueError(f"unknown architecture {arch!r}")


def arch_of(net) -> tuple[str, dict]:
    from ..models.cpsam import CPSAM

    if isinstance(net, CPSAM):
        e = net.encoder
        return "cpsam", dict(dim=e.patch_embed.proj.weight.shape[0], depth=len(e.blocks),
                             heads=e.blocks[0].attn.num_heads, ps=net.ps, bsize=net.bsize, nout=net.nout,
                             rdrop=net.rdrop)
    return "cpnet", dict(nbase=tuple(net.nbase), nout=net.nout, sz=net.sz, norm=net.norm_kind, style_on=net.style_on)


def save_checkpoint(path: str | Path, net) -> None:
    arch, kw = arch_of(net)
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    tmp = p.with_name(p.name + ".tmp")
    torch.save({"arch": arch, "arch_kwargs": kw, "state_dict": {k: v.detach().cpu() for k, v in net.state_dict().items()}},
               tmp)
    os.replace(tmp, p)


def load_checkpoint(path: str | Path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and "arch" in sd:
        net = new_net(sd["arch"], sd.get("arch_kwargs"))
        net.load_state_dict(sd["state_dict"])
        return net
    raise ValueError(f"{path} is not a bioengine cellpose checkpoint (expected arch + state_dict)")


def _load_plain(net, path: str) -> None:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd:
        sd = sd["state_dict"]
    missing, unexpected = net.load_state_dict(sd, strict=False)
    real_missing = [k for k in missing if not k.endswith(("W2", "diam_labels", "diam_mean"))]
    if real_missing:
        raise ValueError(f"weights at {path} do not fit the architecture (missing {real_missing[:5]})")


def build_builtin(name: str, cpsam_arch: str = "vit_l", seed: int = 0):
    """(net, weights) for a built-in model; weights is the loaded path or ``"random"``."""
    if name not in BUILTIN_MODELS:
        raise ValueError(f"'{name}' is not a built-in model ({', '.join(BUILTIN_MODELS)})")
    if name == "cpsam":
        net = new_net("cpsam", CPSAM_ARCHS[cpsam_arch])
    else:
        net = new_net("cpnet")
    path = os.environ.get(WEIGHTS_ENV[name])
    if path and Path(path).exists():
        _load_plain(net, path)
        return net, path
    net.randomize_(seed)
    return net, "random"


def resolve_net(model_id: str, sessions_root: Path, cpsam_arch: str = "vit_l"):
    """(net, weights_source) for a built-in name, a session id, or a checkpoint / weights path."""
    if model_id in BUILTIN_MODELS:
        return build_builtin(model_id, cpsam_arch)
    sid = Path(str(model_id).replace("\\", "/").removesuffix("/status.json")).name
    ck = Path(sessions_root) / sid / "models" / "model"
    if ck.exists():
        return load_checkpoint(ck), f"session:{sid}"
    p = Path(model_id)
    if p.is_file():
        try:
            return load_checkpoint(p), str(p)
        except ValueError:
            net = new_net("cpsam", CPSAM_ARCHS[cpsam_arch])
            _load_plain(net, str(p))
            return net, str(p)
    raise ValueError(f"Model identifier '{model_id}' is not a known pretrained model or a valid session ID / "
                     "published artifact reference.")
