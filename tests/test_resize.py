"""Bilinear resize (diameter rescaling) vs torch F.interpolate(bilinear, align_corners=False)."""
import pytest
import torch
import torch.nn.functional as F

from bioengine_worker_amd.ops.resize import resize_bilinear


def test_resize_cpu_is_interpolate():
    x = torch.rand(2, 3, 37, 53)
    assert torch.equal(resize_bilinear(x, (64, 40)), F.interpolate(x, size=(64, 40), mode="bilinear", align_corners=False))


@pytest.mark.gpu
@pytest.mark.parametrize("size", [(512, 512), (333, 271), (90, 1000), (1, 7)])
def test_resize_gpu_matches_torch(gpu, size):
    g = torch.Generator().manual_seed(sum(size))
    x = torch.rand(2, 3, 200, 300, generator=g) * 100
    ref = F.interpolate(x, size=size, mode="bilinear", align_corners=False)
    got = resize_bilinear(x.to(gpu), size).cpu()
    assert (got - ref).abs().max().item() < 1e-4


@pytest.mark.gpu
def test_tile_queue_chunks_match_one_launch(gpu):
    """Tiles pushed through the network in HBM-budget launches give the one-launch result."""
    from bioengine_worker_amd.cellpose.pipeline import CellposeRunner, EvalParams, synthetic_cells

    runner = CellposeRunner(device=gpu, seed=0)
    img = torch.from_numpy(synthetic_cells(1, 600, 500, nchan=2, ncells=20, seed=1)).to(gpu)
    p = EvalParams(niter=200)
    x = runner._normalize(img.float())
    y1, s1 = runner.run_net(x, p)
    p.max_tiles = 3  # 12 tiles -> 4 launches
    y2, s2 = runner.run_net(x, p)
    torch.cuda.synchronize()
    assert (y1 - y2).abs().max().item() <= 1e-2 * y1.abs().max().item()
    assert runner.tile_budget(EvalParams()) > 1000  # an MI355X holds thousands of 224^2 tiles
