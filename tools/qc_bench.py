"""Flow-QC diffusion time on the headline batch's candidate masks (random-init CPnet, 32 synthetic
512x512 images, ~212 candidates per image): masks_to_flows_gpu per BE_DIFFUSE_VARIANT."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bioengine_worker_amd.cellpose import gpu as cg  # noqa: E402
from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells  # noqa: E402

dev = torch.device("cuda", 0)
runner = CellposeRunner(device=dev, seed=0)
imgs = torch.from_numpy(synthetic_cells(32, 512, 512, nchan=2, seed=0)).to(dev)
p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15)
y, _ = runner.run_net(runner._normalize(imgs.float()), p)
M, nlab = cg.follow_and_label(y, 200, 0.0, 0.4, with_bound=True)
res = {}
ref = None
for v in sys.argv[1:] or ["0", "3"]:
    os.environ["BE_DIFFUSE_VARIANT"] = v
    for _ in range(2):
        mu, err, _ = cg.masks_to_flows_gpu(M, dp=y, nlab=nlab)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t = time.perf_counter()
        mu, err, _ = cg.masks_to_flows_gpu(M, dp=y, nlab=nlab)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    if ref is None:
        ref = mu.clone()
    res[v] = {"ms": round(ts[5], 3), "identical_to_first": bool(torch.equal(mu, ref))}
print(json.dumps(res))
