#!/usr/bin/env python3
"""CPnet inference engine, whole network, one headline batch (288 tiles of 224x224 = 32 images of
512x512), under engine configurations built in one process (A/B of the conv paths):
baseline per-layer deep levels, igemm / ping-pong (gemm_pp) deep levels, either also at level 1
(pairs at level 0 only).
HIP-event median of --reps forwards; relative RMS of each config's output against the baseline."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

CONFIGS = {
    "default": {},
    "perlayer_deep": {"BE_CPNET_IGEMM": "0", "BE_CPNET_PAIR_LEVELS": "0,1"},
    "perlayer_L1": {"BE_CPNET_IGEMM": "0", "BE_CPNET_PAIR_LEVELS": "0"},
    "igemm_deep": {"BE_CPNET_IGEMM": "1", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_IGEMM_LEVELS": "2,3"},
    "igemm_deep_L1": {"BE_CPNET_IGEMM": "1", "BE_CPNET_PAIR_LEVELS": "0", "BE_CPNET_IGEMM_LEVELS": "1,2,3"},
    "igemm_L3": {"BE_CPNET_IGEMM": "1", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_IGEMM_LEVELS": "3"},
    "pp_deep": {"BE_CPNET_IGEMM": "pp", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_IGEMM_LEVELS": "2,3"},
    "pp_deep_L1": {"BE_CPNET_IGEMM": "pp", "BE_CPNET_PAIR_LEVELS": "0", "BE_CPNET_IGEMM_LEVELS": "1,2,3"},
    "pp_deep_cfg0": {"BE_CPNET_IGEMM": "pp", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_PP_CFG": "0",
                     "BE_CPNET_IGEMM_LEVELS": "2,3"},
    "pp_deep_cfg1": {"BE_CPNET_IGEMM": "pp", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_PP_CFG": "1",
                     "BE_CPNET_IGEMM_LEVELS": "2,3"},
    "pp_deep_cfg2": {"BE_CPNET_IGEMM": "pp", "BE_CPNET_PAIR_LEVELS": "0,1", "BE_CPNET_PP_CFG": "2",
                     "BE_CPNET_IGEMM_LEVELS": "2,3"},
}
KEYS = sorted({k for env in CONFIGS.values() for k in env})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", type=int, default=288)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    a = ap.parse_args()
    from bioengine_worker_amd.models.cpnet import CPnet, CPnetEngine

    dev = torch.device("cuda", 0)
    net = CPnet().randomize_(0).eval()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.zeros(a.tiles, 224, 224, 8, device=dev, dtype=torch.bfloat16)
    x[..., :2] = torch.randn(a.tiles, 224, 224, 2, device=dev, generator=g).to(torch.bfloat16)
    base = None
    for name in a.configs.split(","):
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(CONFIGS[name])
        eng = CPnetEngine(net, dev)
        y, _ = eng(x)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng(x)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        row = {"config": name, "ms": round(ts[len(ts) // 2], 3), "min_ms": round(ts[0], 3),
               "igemm_layers": len(eng.ig), "pairs": len(eng.pair)}
        if base is None:
            base = y.float()
        else:
            row["rel_rms_vs_perlayer"] = round(((y.float() - base).pow(2).mean().sqrt() /
                                                base.pow(2).mean().sqrt()).item(), 5)
        print(json.dumps(row), flush=True)
        del eng, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
