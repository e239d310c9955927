"""Snapshot-sharded sequence on the HIP path: two ranks sharing cuda:0 (gloo, host-staged collectives)
against the unsharded HIP model on the same sequence and weights (fp32, dropout 0)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

COUNTS = [40, 57, 33, 57, 49, 21]


def _setup(dev):
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(node_feature_dim=8, edge_feature_dim=0, hidden_dim=64, num_heads=4, num_layers=2,
                      dropout=0.0, output_dim=1, window_size=3)
    torch.manual_seed(21)
    model = TAGAN(cfg).to(dev)
    g = torch.Generator().manual_seed(4)
    seq = []
    for n in COUNTS:
        seq.append((torch.randn(n, 8, generator=g).to(dev), torch.randint(0, n, (2, 4 * n), generator=g).to(dev),
                    None, list(range(n))))
    return model, seq


def _worker(rank, world, store_path, results):
    # a file rendezvous: no TCP port to race for with another test's lingering store
    dist.init_process_group("gloo", init_method="file://" + store_path, rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
    labels = torch.tensor([1.0], device=dev)
    if rank == 0:
        ref_model, seq = _setup(dev)
        ref = ref_model(seq, labels)
        ref["loss"].backward()
        results["ref_loss"] = float(ref["loss"])
        results["ref_grads"] = {k: p.grad.cpu() for k, p in ref_model.named_parameters() if p.grad is not None}
    model, seq = _setup(dev)
    sharded = SnapshotShardedTAGAN.for_model(model)
    t0, t1 = blocks(len(COUNTS), world)[rank]
    out = sharded(seq[t0:t1], COUNTS, labels)
    out["loss"].backward()
    ShardGradSync(list(model.named_parameters())).sync()
    torch.cuda.synchronize()
    results["loss%d" % rank] = float(out["loss"])
    results["grads%d" % rank] = {k: p.grad.cpu() for k, p in model.named_parameters() if p.grad is not None}
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_hip_matches_unsharded():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tempfile
    store_path = os.path.join(tempfile.mkdtemp(prefix="tagan_shard_"), "store")
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, store_path, res), nprocs=2, join=True)
        res = dict(res)
    ref = res["ref_grads"]
    for r in range(2):
        assert abs(res["loss%d" % r] - res["ref_loss"]) < 1e-5
        got = res["grads%d" % r]
        assert sorted(got) == sorted(ref)
        for k, g in ref.items():
            err = float((got[k] - g).abs().max())
            assert err <= 1e-4 + 1e-4 * float(g.abs().max()), (r, k, err)   # north_star 1e-4
