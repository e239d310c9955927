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


def _worker_c2(rank, world, store_path, results):
    """The C2 workload (10k nodes, 100k Zipf edges per snapshot, 32 snapshots, H 128, 8 heads; dropout 0) sharded by
    snapshot over two ranks on one GPU, against the unsharded model run by rank 0 -- the stream-GEMM / LN-fused
    blocks at full C2 size through the all-to-all and the pooling all-reduce."""
    dist.init_process_group("gloo", init_method="file://" + store_path, rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
    cfg = synthetic.config_for("c2", dropout=0.0)
    seq = synthetic.make_sequence("c2", dev, seed=77)
    counts = [int(x.shape[0]) for x, _, _, _ in seq]
    labels = torch.tensor([1.0], device=dev)
    if rank == 0:
        torch.manual_seed(5)
        ref_model = TAGAN(cfg).to(dev)
        ref = ref_model(seq, labels=labels)
        ref["loss"].backward()
        results["ref_loss"] = float(ref["loss"])
        results["ref_grads"] = {k: p.grad.cpu() for k, p in ref_model.named_parameters() if p.grad is not None}
        del ref_model, ref
    torch.manual_seed(5)
    model = TAGAN(cfg).to(dev)
    sharded = SnapshotShardedTAGAN.for_model(model)
    t0, t1 = blocks(len(seq), world)[rank]
    out = sharded(seq[t0:t1], counts, labels)
    out["loss"].backward()
    ShardGradSync(list(model.named_parameters())).sync()
    torch.cuda.synchronize()
    results["loss%d" % rank] = float(out["loss"])
    results["grads%d" % rank] = {k: p.grad.cpu() for k, p in model.named_parameters() if p.grad is not None}
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_hip_matches_unsharded_c2():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tempfile
    from golden_io import assert_close
    store_path = os.path.join(tempfile.mkdtemp(prefix="tagan_shard_c2_"), "store")
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker_c2, args=(2, store_path, res), nprocs=2, join=True)
        res = dict(res)
    ref = res["ref_grads"]
    for r in range(2):
        assert abs(res["loss%d" % r] - res["ref_loss"]) <= 1e-5 * max(1.0, abs(res["ref_loss"]))
        got = res["grads%d" % r]
        assert sorted(got) == sorted(ref)
        for k, g in ref.items():
            # north_star 1e-4 elementwise (relative to the tensor's scale) + the suite's normwise gradient bound
            assert_close("grad." + k, got[k], g, atol=1e-4 * max(1.0, float(g.abs().max())), rtol=1e-4)


# C5 geometry (BASELINE configs[4]: T = 128 snapshots, hidden 256, 16 heads) with the node count reduced so that the
# unsharded reference and two sharded ranks fit one GPU together; edges keep the C5 degree (20 per node).
C5_NODES, C5_EDGES = 6000, 120_000
C5_SAMPLE = 256


def _worker_c5(rank, world, store_path, results):
    """The C5-geometry sequence sharded by snapshot over two ranks on one GPU (gloo): each rank runs the geometric
    stage on its 64 snapshots (H = 256 stream GEMMs), the all-to-all to node rows, the v5 temporal kernel (T = 128,
    d = 16) on its N / 2 row slice, the pooling all-reduce and the flagged gradient sync; rank 0 also runs the
    unsharded model.  Each rank's temporal block is checked on sampled rows of its slice against the fp64 oracle
    (forward, and the input gradient for a unit upstream gradient on those rows).  Then bench.c5_shard_record
    drives the same step through the bench's measurement path once."""
    dist.init_process_group("gloo", init_method="file://" + store_path, rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import tagan_amd  # noqa: F401
    import oracle
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
    cfg = synthetic.config_for("c5", dropout=0.0)
    T, heads = synthetic.CONFIGS["c5"][2], synthetic.CONFIGS["c5"][4]
    full = synthetic.make_sequence("c5", dev, seed=91, nodes=C5_NODES, edges=C5_EDGES)
    counts = [int(x.shape[0]) for x, _, _, _ in full]
    labels = torch.tensor([1.0], device=dev)
    if rank == 0:
        torch.manual_seed(5)
        ref_model = TAGAN(cfg).to(dev)
        ref = ref_model(full, labels=labels)
        ref["loss"].backward()
        results["ref_loss"] = float(ref["loss"])
        results["ref_grads"] = {k: p.grad.cpu() for k, p in ref_model.named_parameters() if p.grad is not None}
        del ref_model, ref
        torch.cuda.empty_cache()
    t0, t1 = blocks(T, world)[rank]
    seq = synthetic.take(full, t0, t1)
    del full
    torch.manual_seed(5)
    model = TAGAN(cfg).to(dev)
    sharded = SnapshotShardedTAGAN.for_model(model)
    cap = {}
    temporal = sharded.temporal

    def probe(xt):   # the rank's temporal block: keep its input and output for the oracle check
        xt.retain_grad()
        out = temporal(xt)
        out.retain_grad()
        cap["x"], cap["out"] = xt, out
        return out
    sharded.temporal = probe
    out = sharded(seq, counts, labels)
    out["loss"].backward()
    ShardGradSync(list(model.named_parameters())).sync()
    torch.cuda.synchronize()
    results["loss%d" % rank] = float(out["loss"])
    results["grads%d" % rank] = {k: p.grad.cpu() for k, p in model.named_parameters() if p.grad is not None}
    # sampled rows of this rank's slice vs the fp64 oracle (shipped mask: ones(T, T), causal iff T == heads)
    x, o = cap["x"], cap["out"]
    n_r = x.shape[1]
    gen = torch.Generator().manual_seed(17 + rank)
    rows = torch.unique(torch.cat([torch.randint(0, n_r, (C5_SAMPLE,), generator=gen), torch.tensor([n_r - 1])]))
    ta = model.temporal_attention
    P = {"temporal_attention." + k: v.detach().cpu().double().requires_grad_(v.is_floating_point())
         for k, v in ta.state_dict().items()}
    x64 = x.detach()[:, rows.to(dev)].permute(1, 0, 2).cpu().double().requires_grad_(True)
    ref_o = oracle.temporal_attention(x64, P, "temporal_attention", heads, cls="asym", causal=cfg.causal_attention,
                                      relative_position_bias=cfg.asymmetric_temporal_bias,
                                      asymmetric_window_size=cfg.window_size, attention_mask=torch.ones(T, T))
    got_o = o.detach()[:, rows.to(dev)].permute(1, 0, 2).cpu().double()
    results["temporal_out_err%d" % rank] = float((got_o - ref_o).abs().max() / ref_o.abs().max())
    # the upstream gradient the rank's block received on those rows (pooling + head backward), through the oracle
    go = o.grad.detach()[:, rows.to(dev)].permute(1, 0, 2).cpu().double()
    (ref_o * go).sum().backward()
    gx = x.grad.detach()[:, rows.to(dev)].permute(1, 0, 2).cpu().double()
    results["temporal_dx_err%d" % rank] = float((gx - x64.grad).norm() / x64.grad.norm())
    results["rows%d" % rank] = int(rows.numel())
    del out, cap, x, o, seq, model, sharded
    torch.cuda.empty_cache()
    import bench
    rec = bench.c5_shard_record(dev, rank, world, None, "gloo", steps=1, warmup=1, nodes=C5_NODES, edges=C5_EDGES)
    results["record%d" % rank] = dict(rec)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_sharded_hip_matches_unsharded_c5_geometry():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tempfile
    from golden_io import assert_close
    store_path = os.path.join(tempfile.mkdtemp(prefix="tagan_shard_c5_"), "store")
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker_c5, args=(2, store_path, res), nprocs=2, join=True)
        res = dict(res)
    ref = res["ref_grads"]
    for r in range(2):
        assert abs(res["loss%d" % r] - res["ref_loss"]) <= 1e-5 * max(1.0, abs(res["ref_loss"]))
        got = res["grads%d" % r]
        assert sorted(got) == sorted(ref)
        for k, g in ref.items():
            assert_close("grad." + k, got[k], g, atol=1e-4 * max(1.0, float(g.abs().max())), rtol=1e-4)
        assert res["rows%d" % r] >= C5_SAMPLE // 2
        assert res["temporal_out_err%d" % r] <= 1e-5, res["temporal_out_err%d" % r]
        assert res["temporal_dx_err%d" % r] <= 1e-4, res["temporal_dx_err%d" % r]
        rec = res["record%d" % r]
        assert rec["parallelism"] == "snapshot-shard2" and rec["scaling"] == "strong" and rec["n_ranks"] == 2
        assert rec["value"] > 0 and rec["ms_per_step"] > 0
        assert set(rec["exchange_ms_per_step"]) >= {"all_to_all", "pool_allreduce", "grad_allreduce"}
