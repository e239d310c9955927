"""Snapshot-sharded single-sequence mode (tagan_amd.sharded) on CPU with gloo, world sizes 2 and 3.

The stage functions are wired to the CPU oracle (test infrastructure), so these tests check the
exchange logic — snapshot→row all-to-all and its reverse, pooling partials + all-reduce, the
replicated head, the SUM vs SUM/P gradient exchange — against the unsharded oracle forward of the
same sequence.  On the GPU the same class is wired to the HIP model (``for_model``).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from oracle.tagan_oracle import _lin, _ln, bce_loss, classification_head, graph_attention, temporal_attention

H, HEADS, T, W = 16, 2, 5, 5
COUNTS = [9, 13, 7, 13, 11]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _params():
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(node_feature_dim=6, edge_feature_dim=0, hidden_dim=H, num_heads=HEADS, num_layers=2,
                      dropout=0.0, output_dim=1, window_size=W)
    torch.manual_seed(5)
    sd = TAGAN(cfg).state_dict()
    return cfg, {k: v.detach().clone().double().requires_grad_(v.dtype.is_floating_point) for k, v in sd.items()}


def _sequence():
    g = torch.Generator().manual_seed(11)
    seq = []
    for n in COUNTS:
        x = torch.randn(n, 6, generator=g, dtype=torch.float64)
        ei = torch.randint(0, n, (2, 3 * n), generator=g)
        seq.append((x, ei, None, list(range(n))))
    return seq


def _stage_fns(P):
    def encode(snaps):
        outs = []
        for x, ei, _, _ in snaps:
            h = _lin(x, P, "node_embedding")
            skip = h
            for i in range(2):
                h = graph_attention(h, ei, P, "geometric_attention_layers.%d" % i, HEADS, "euclidean", True, False,
                                    mode="sparse")
                if i == 0:
                    h = h + _ln(skip, P, "skip_layer_norm")
            outs.append(h)
        return torch.cat(outs, 0), [int(o.shape[0]) for o in outs]

    def temporal(xt):
        out = temporal_attention(list(xt.unbind(0)), P, "temporal_attention", HEADS, cls="asym", causal=False,
                                 use_layer_norm=True, relative_position_bias=True, asymmetric_window_size=W,
                                 attention_mask=torch.ones(T, T, dtype=xt.dtype))
        return out.transpose(0, 1)

    def head(pooled, labels):
        logits = classification_head(pooled.unsqueeze(0), P, True)
        return {"logits": logits, "loss": bce_loss(logits, labels)}

    return encode, temporal, head


def _worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
    cfg, P = _params()
    seq = _sequence()
    labels = torch.tensor([1.0], dtype=torch.float64)
    if rank == 0:   # unsharded reference on rank 0
        _, Pref = _params()
        ref = oracle.tagan_forward(Pref, dict(hidden_dim=H, num_heads=HEADS, num_layers=2, output_dim=1,
                                              window_size=W), seq, labels)
        ref["loss"].backward()
        results["ref_loss"] = ref["loss"].detach()
        results["ref_grads"] = {k: v.grad.clone() for k, v in Pref.items() if v.grad is not None}
    enc, tmp, head = _stage_fns(P)
    model = SnapshotShardedTAGAN(enc, tmp, head)
    t0, t1 = blocks(T, world)[rank]
    out = model(seq[t0:t1], COUNTS, labels)
    out["loss"].backward()
    ShardGradSync(list(P.items())).sync()
    results["loss%d" % rank] = out["loss"].detach()
    results["grads%d" % rank] = {k: v.grad.clone() for k, v in P.items() if v.grad is not None}
    results["none%d" % rank] = sorted(k for k, v in P.items() if v.requires_grad and v.grad is None)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sequence_matches_unsharded(world):
    port = _free_port()
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(world, port, res), nprocs=world, join=True)
        res = dict(res)
    ref_loss, ref_grads = res["ref_loss"], res["ref_grads"]
    for r in range(world):
        assert torch.allclose(res["loss%d" % r], ref_loss, atol=1e-12, rtol=1e-10), r
        got = res["grads%d" % r]
        assert sorted(got) == sorted(ref_grads), (r, set(got) ^ set(ref_grads))
        for k, g in ref_grads.items():
            assert torch.allclose(got[k], g, atol=1e-10, rtol=1e-8), (r, k, float((got[k] - g).abs().max()))
        assert res["none%d" % r] == res["none0"]


def test_pool_partial_sums_to_reference_pooling():
    from tagan_amd.sharded import blocks, pool_partial
    g = torch.Generator().manual_seed(0)
    for T_, N_, P_ in [(5, 13, 2), (7, 4, 3), (4, 4, 4), (3, 10, 1)]:
        out = torch.randn(T_, N_, 8, generator=g, dtype=torch.float64)
        want = out.transpose(0, 1).reshape(T_, N_, 8).mean(1)          # TAGAN._pool
        got = sum(pool_partial(out[:, a:b], a, N_) for a, b in blocks(N_, P_)) / N_
        assert torch.allclose(got, want, atol=1e-12)
