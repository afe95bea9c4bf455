"""Census of the candidate masks the headline batch feeds to flow QC (random-init CPnet on synthetic
images): per-image count, size and box distribution, niter, and how the diffusion buckets fill."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bioengine_worker_amd.cellpose import gpu as cg  # noqa: E402
from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells  # noqa: E402

dev = torch.device("cuda", 0)
runner = CellposeRunner(device=dev, seed=0)
imgs = torch.from_numpy(synthetic_cells(32, 512, 512, nchan=2, seed=0)).to(dev)
p = EvalParams(niter=200, flow_threshold=0.4, cellprob_threshold=0.0, min_size=15)
x = runner._normalize(imgs.float())
y, _ = runner.run_net(x, p)
M, nlab = cg.follow_and_label(y, 200, 0.0, 0.4, with_bound=True)
counts = cg.label_counts(M, nlab).cpu()
bbox = cg.mask_bboxes(M, nlab).cpu()
valid = (counts > 0)
ly = (bbox[..., 1] - bbox[..., 0] + 1).clamp(min=0)
lx = (bbox[..., 3] - bbox[..., 2] + 1).clamp(min=0)
area = (ly + 2) * (lx + 2)
cnt = counts[valid].float()
print(json.dumps({
    "masks": int(valid.sum()), "per_image": round(float(valid.sum()) / 32, 1),
    "lt_min_size": int(((counts > 0) & (counts < 15)).sum()),
    "px_quantiles": [float(q) for q in torch.quantile(cnt, torch.tensor([0.1, 0.5, 0.9, 0.99]))],
    "max_box": [int(ly[valid].max()), int(lx[valid].max())],
    "niter_img": (2 * (ly + lx + 2) * valid).max(1).values.tolist(),
    "box_area_sum_by_bucket": {str(c): int(area[valid & (16 * area <= c)].sum()) for c in [6144, 12288, 24576, 49152, 81920, 159744]},
    "fill_frac_of_box": round(float(cnt.sum() / area[valid].float().sum()), 3),
}))
