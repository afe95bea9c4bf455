#!/usr/bin/env python3
"""Sanitizer builds of the C++ host runtime (``csrc/runtime/*.cpp``) + its self-test driver.

Builds ``csrc/runtime/tests/runtime_selftest.cpp`` together with every runtime source under

* ``asan``  — ``-fsanitize=address,undefined -fno-sanitize-recover=all`` (heap/stack overflows,
  use-after-free, leaks, signed overflow, misaligned access...),
* ``tsan``  — ``-fsanitize=thread`` (data races between the ring's producer and consumer threads),

and runs each.  Host code only: GPU-side sanitizers are not available on the MI355X pool, and the
HIP kernels are covered by their PyTorch-oracle numerics tests instead.
Usage: ``python tools/sanitize_runtime.py [asan|tsan ...]``; exit status != 0 on any finding.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
RT = ROOT / "csrc" / "runtime"
OUT = ROOT / "build" / "sanitize"

MODES = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}
ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1",
             "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"},
}


def build(mode: str) -> Path:
    cxx = shutil.which("g++") or "g++"
    OUT.mkdir(parents=True, exist_ok=True)
    exe = OUT / f"runtime_selftest_{mode}"
    srcs = sorted(RT.glob("*.cpp")) + [RT / "tests" / "runtime_selftest.cpp"]
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-pthread", *MODES[mode], *map(str, srcs), "-o", str(exe), "-lrt"]
    subprocess.run(cmd, check=True)
    return exe


def run(mode: str) -> int:
    exe = build(mode)
    env = dict(os.environ, **ENV[mode])
    env.pop("LD_PRELOAD", None)  # sanitizer runtimes must be first in the initial library list
    args = [str(exe)]
    if mode == "tsan":
        args.append("--no-fork")  # TSan does not follow fork()ed children; the asan run covers it
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=300)
    sys.stdout.write(f"[{mode}] rc={r.returncode}\n{r.stdout}{r.stderr[-4000:]}")
    return r.returncode


def main(argv=None) -> int:
    modes = (argv if argv is not None else sys.argv[1:]) or list(MODES)
    return max(run(m) for m in modes)


if __name__ == "__main__":
    sys.exit(main())
