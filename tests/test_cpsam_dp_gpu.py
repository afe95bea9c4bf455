"""The data-parallel CPSAM step path on one GPU (1-rank RCCL group, ``force_dp_path``): fwd+bwd
captured as a chain of HIP graphs cut at gradient-bucket boundaries, each bucket's all-reduce issued
between segment replays.  It must reproduce the single-GPU graph step."""
import socket

import pytest
import torch
import torch.distributed as dist


@pytest.mark.gpu
def test_cpsam_segmented_dp_graph_matches_single_gpu_graph(gpu):
    from bioengine_worker_amd.cellpose.model_store import CPSAM_ARCHS, new_net
    from bioengine_worker_amd.train.cellpose_train import CellposeTrainer, TrainConfig

    def net():
        m = new_net("cpsam", dict(CPSAM_ARCHS["tiny"], bsize=256))  # rel-pos attention: 32 x 32 token grid
        torch.manual_seed(0)
        for p in m.parameters():
            p.data.normal_(0, 0.05) if p.dim() > 1 else p.data.normal_(0, 0.01)
        m.rdrop = 0.0
        return m

    g = torch.Generator().manual_seed(3)
    B, S = 2, 256
    xs = [torch.randn(B, 3, S, S, generator=g).to(gpu) for _ in range(4)]
    ls = []
    for _ in range(4):
        lbl = torch.zeros(B, 3, S, S)
        lbl[:, 0] = (torch.rand(B, S, S, generator=g) > 0.6).float()
        lbl[:, 1:] = 0.3 * torch.randn(B, 2, S, S, generator=g)
        ls.append(lbl.to(gpu))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=gpu)
    try:
        flats, losses = [], []
        for force in (False, True):
            cfg = TrainConfig(batch_size=B, bsize=S, lr=1e-3, weight_decay=1e-4, bucket_mb=0.05, force_dp_path=force)
            tr = CellposeTrainer(net(), cfg, gpu)
            assert tr.ar.active == force
            ll = [float(tr._step_cpsam(x, l)) for x, l in zip(xs, ls)]
            if force:
                segs = tr._cpsam_dp[1]
                assert len(segs) > 3 and not tr._cpsam_graph_failed  # several bucket cut points
            flats.append(tr.fp.flat.detach().clone())
            losses.append(ll)
    finally:
        dist.destroy_process_group()
    torch.testing.assert_close(flats[1], flats[0], rtol=1e-5, atol=1e-6)
    assert losses[0] == pytest.approx(losses[1], rel=1e-5)
