#!/usr/bin/env python3
"""Build the native libraries of bioengine_worker_amd in-tree.

* ``libbe_hip.so``     — every ``csrc/kernels/*.hip`` compiled with ``hipcc --offload-arch=gfx950``
  (CDNA4 only; no other targets, no CUDA, no hipify).
* ``libbe_runtime.so`` — the host runtime in ``csrc/runtime/*.cpp`` (cross-process shared-memory
  SPSC ring used as the router <-> replica bulk-data lane, serial EM post-processing: priority-flood
  watershed and peak spacing) compiled with g++; it has no GPU dependency so it also runs in
  CPU-only CI.  ``tools/sanitize_runtime.py`` builds the same sources under ASan/UBSan and TSan.

Objects are cached under ``build/`` keyed by source mtime + flags, so rebuilding after editing one
kernel recompiles only that file.  Usage: ``python tools/build_native.py [--only hip|runtime] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OUT_DIR = ROOT / "bioengine_worker_amd" / "_native"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("BE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_lib_dir() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec is None or spec.origin is None:
            return None
        return str(Path(spec.origin).parent / "lib")
    except Exception:
        return None


HIP_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
    "-I",
    str(CSRC / "kernels"),
]
# Per-source extra flags.  clahe: OpenCV bit parity needs separately rounded fp32 products; hipcc's
# default contraction fuses them into FMAs even under `#pragma clang fp contract(off)`.
# attention: MFMA accumulators in arch VGPRs (the default AGPR form moved every S / O tile through
# v_accvgpr_read/write around the softmax: 192 moves per KV tile); forward 0.085 -> 0.076 ms at B=8.
# gemm_mt: same, and without it hipcc shuffles the accumulators through a scratch AGPR quad every MFMA.
# conv_pair: no SLP vectorisation -- packed-f32 VALU (v_pk_fma_f32) issued beside another wave's
# MFMAs is slow on CDNA4; the ping-pong half-blocks run their VALU phases exactly there
# (profiles/r05/conv/pp_noslp_ab: stem -18 %, 32->32 -7.5 %, 64->32 up -9 %, headline +1.5 %)
PER_SOURCE_FLAGS = {"clahe": ["-ffp-contract=off"], "attention": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
                    "gemm_mt": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"], "conv_pair": ["-fno-slp-vectorize"]}
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread", "-I", str(CSRC / "runtime")]


def _key(src: Path, flags: list[str]) -> str:
    h = hashlib.sha1()
    h.update(" ".join(flags).encode())
    h.update(src.read_bytes())
    for hdr in sorted(list(src.parent.glob("*.h")) + list(src.parent.glob("*.inc"))):
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def _compile(cmd_base: list[str], src: Path, flags: list[str]) -> Path:
    obj = BUILD / f"{src.stem}.{_key(src, flags)}.o"
    if obj.exists():
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = cmd_base + flags + ["-c", str(src), "-o", str(obj) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {src}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


_PROTO = None


def extract_signatures(srcs) -> dict[str, str]:
    """Parse ``extern "C"`` entry points ``int be_*(...)`` and map each parameter to a ctypes code:
    pointer -> p, hipStream_t -> s, float -> f, long long/int64 -> l, int -> i."""
    import re

    sigs = {}
    pat = re.compile(r"\bint\s+(be_[A-Za-z0-9_]+)\s*\(([^)]*)\)\s*\{", re.S)
    for src in srcs:
        text = Path(src).read_text()
        for m in pat.finditer(text):
            name, params = m.group(1), m.group(2).strip()
            codes = []
            if params and params != "void":
                for prm in params.split(","):
                    prm = " ".join(prm.split())
                    if "*" in prm:
                        codes.append("p")
                    elif "hipStream_t" in prm:
                        codes.append("s")
                    elif prm.startswith("float") or prm.startswith("const float"):
                        codes.append("f")
                    elif prm.startswith("double"):
                        codes.append("d")
                    elif "long long" in prm or "int64_t" in prm:
                        codes.append("l")
                    else:
                        codes.append("i")
            sigs[name] = "".join(codes)
    return sigs


def build_hip(jobs: int, variant: str | None = None, vsrc: str | None = None, vflags: list[str] | None = None) -> Path:
    """``variant``: build ``_native/variants/<variant>/libbe_hip.so`` with ``vflags`` added to the
    sources whose stem contains ``vsrc`` (kernel tuning experiments; load with BE_HIP_LIB=...)."""
    srcs = sorted((CSRC / "kernels").glob("*.hip"))
    if not srcs:
        raise RuntimeError("no HIP sources")

    def flags_for(src):
        base = HIP_FLAGS + PER_SOURCE_FLAGS.get(src.stem, [])
        if variant and vsrc and vsrc in src.stem:
            return base + list(vflags or [])
        return base

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile([HIPCC], s, flags_for(s)), srcs))
    out = OUT_DIR / "libbe_hip.so"
    if variant:
        out = OUT_DIR / "variants" / variant / "libbe_hip.so"
        out.parent.mkdir(parents=True, exist_ok=True)
    tl = _torch_lib_dir()
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out) + ".tmp"] + [str(o) for o in objs]
    if tl and Path(tl, "libamdhip64.so").exists():
        # Resolve libamdhip64 against the runtime PyTorch ships so the process has ONE HIP runtime.
        link += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("link failed: libbe_hip.so")
    os.replace(str(out) + ".tmp", out)
    import json

    (out.parent / "hip_signatures.json").write_text(json.dumps(extract_signatures(srcs), indent=1, sort_keys=True))
    return out


def build_runtime(jobs: int) -> Path | None:
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    if not srcs:
        return None
    cxx = shutil.which("g++") or "g++"
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile([cxx], s, CXX_FLAGS), srcs))
    out = OUT_DIR / "libbe_runtime.so"
    r = subprocess.run([cxx, "-shared", "-fPIC", "-pthread", "-o", str(out) + ".tmp"] + [str(o) for o in objs] + ["-lrt"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("link failed: libbe_runtime.so")
    os.replace(str(out) + ".tmp", out)
    import json

    (OUT_DIR / "runtime_signatures.json").write_text(json.dumps(extract_signatures(srcs), indent=1, sort_keys=True))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["hip", "runtime"], default=None)
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--variant", default=None, help="tuning variant name (writes _native/variants/NAME)")
    ap.add_argument("--vsrc", default=None, help="source stem substring the variant flags apply to")
    ap.add_argument("--vflags", default="", help="extra hipcc flags of the variant, e.g. '-DCONV_X=1'")
    args = ap.parse_args(argv)
    if args.variant:
        print(f"built {build_hip(args.jobs, args.variant, args.vsrc, args.vflags.split())}")
        return 0
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    if args.only in (None, "runtime"):
        p = build_runtime(args.jobs)
        print(f"built {p}")
    if args.only in (None, "hip"):
        p = build_hip(args.jobs)
        print(f"built {p}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
