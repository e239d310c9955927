"""Sequence-level data parallelism on the HIP path (bench.py's multi-rank step, eager form): two ranks sharing
cuda:0 over gloo (device tensors host-staged by distributed.all_reduce_ / broadcast_), each training on its own
sequence, against the mean of the two ranks' gradients computed in one process (fp32, dropout 0)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

COUNTS = [(40, 57, 33, 57), (49, 21, 60, 38)]


def _model(dev):
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(node_feature_dim=8, edge_feature_dim=0, hidden_dim=64, num_heads=4, num_layers=2,
                      dropout=0.0, output_dim=1, window_size=3)
    torch.manual_seed(5)
    return TAGAN(cfg).to(dev).train()


def _seq(rank, dev):
    g = torch.Generator().manual_seed(100 + rank)
    return [(torch.randn(n, 8, generator=g).to(dev), torch.randint(0, n, (2, 4 * n), generator=g).to(dev), None,
             list(range(n))) for n in COUNTS[rank]]


def _worker(rank, world, store_path, static, results):
    dist.init_process_group("gloo", init_method="file://" + store_path, rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from tagan_amd.distributed import GradBucket, broadcast_parameters
    labels = torch.tensor([1.0 if rank == 0 else 0.0], device=dev)
    if rank == 0:   # the reference: both ranks' sequences in one process, gradients averaged
        grads = []
        for r in range(world):
            m = _model(dev)
            out = m(_seq(r, dev), labels=torch.tensor([1.0 if r == 0 else 0.0], device=dev))
            out["loss"].backward()
            grads.append({k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None})
        results["ref"] = {k: sum(g[k] for g in grads) / world for k in grads[0]}
    model = _model(dev)
    with torch.no_grad():   # perturb rank 1's weights: broadcast_parameters must restore rank 0's
        if rank == 1:
            for p in model.parameters():
                p.add_(1.0)
    broadcast_parameters(model)
    bucket = GradBucket(model.parameters())
    out = model(_seq(rank, dev), labels=labels)
    out["loss"].backward()
    bucket.allreduce_mean(static=static)
    torch.cuda.synchronize()
    results["grads%d" % rank] = {k: p.grad.cpu() for k, p in model.named_parameters() if p.grad is not None}
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("static", [False, True])
def test_dp_two_ranks_mean_gradient(static):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tempfile
    store_path = os.path.join(tempfile.mkdtemp(prefix="tagan_dp_"), "store")
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, store_path, static, res), nprocs=2, join=True)
        res = dict(res)
    ref = res["ref"]
    for r in range(2):
        got = res["grads%d" % r]
        assert sorted(got) == sorted(ref)
        for k, g in ref.items():
            err = float((got[k] - g).abs().max())
            assert err <= 1e-4 + 1e-4 * float(g.abs().max()), (r, k, err)   # north_star 1e-4
    for k in ref:   # both ranks hold the same mean gradient
        assert torch.equal(res["grads0"][k], res["grads1"][k]), k
