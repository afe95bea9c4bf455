#!/usr/bin/env python3
"""Per-parameter cosine similarity of the HIP training engine's gradients vs fp32 autograd (GPU)."""
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(B=2, S=64, style_on=True):
    from bioengine_worker_amd.models.cpnet import CPnet
    from bioengine_worker_amd.ops import train_ops
    from bioengine_worker_amd.parallel.ddp import FlatParams
    from bioengine_worker_amd.train.cpnet_engine import CPnetTrainEngine

    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = CPnet(style_on=style_on).randomize_(0).train()
    ref = copy.deepcopy(net).to(gpu)
    x = torch.randn(B, 2, S, S, device=gpu)
    lbl = torch.zeros(B, 3, S, S, device=gpu)
    lbl[:, 0] = (torch.rand(B, S, S, device=gpu) > 0.6).float()
    lbl[:, 1:] = 0.3 * torch.randn(B, 2, S, S, device=gpu)
    loss_ref = train_ops.seg_loss_ref(ref(x)[0], lbl)
    loss_ref.backward()
    net = net.to(gpu)
    fp = FlatParams(net, gpu)
    eng = CPnetTrainEngine(net, fp, B=B, S=S, device=gpu)
    y = eng.forward(x)
    with torch.no_grad():
        yr = ref(x)[0]
    print(json.dumps({"fwd_rel": float((y - yr).abs().max() / yr.abs().max())}))
    loss = eng.loss_and_backward(x, lbl)
    torch.cuda.synchronize()
    print(json.dumps({"loss": float(loss), "loss_ref": float(loss_ref.detach())}))
    nr = dict(ref.named_parameters())
    for name, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g_ref = nr[name].grad.float()
        g = p.grad.float()
        cos = torch.nn.functional.cosine_similarity(g.flatten(), g_ref.flatten(), dim=0).item()
        print(json.dumps({"p": name, "cos": round(cos, 4), "ref_max": float(g_ref.abs().max()),
                          "max": float(g.abs().max())}))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:3]])
