"""Snapshot ingestion on the HIP path: TAGAN.forward on the reference's snapshot DICTS (global user ids,
variable node counts, edge_attr absent or present; model.py:187-230, the format of
preprocess_social_media.py:374-389) against goldens minted from the reference itself
(tests/golden/ingest_dict_*), the packed SnapshotBatch path (host dicts -> pinned staging -> one copy per
array -> tagan_csr_build on the concatenated edges) bitwise equal to the per-snapshot list path, the
deferred edge-index validation, and the device global-id index (model.py:184-201)."""
import pytest
import torch

import golden_io as G

pytestmark = pytest.mark.gpu

OUT_ATOL, OUT_RTOL = 1e-4, 1e-4
GRAD_ATOL, GRAD_RTOL = 1e-4, 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _model(meta, t, dev):
    from tagan_amd import TAGAN, TAGANConfig
    model = TAGAN(TAGANConfig(**dict(meta["config"], device="cuda")))
    model.load_state_dict(G.state_dict(t), strict=True)
    return model.to(dev).train()


def _run(model, seq, labels):
    out = model(seq, labels=labels)
    out["loss"].backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    return out, grads


@pytest.mark.parametrize("case", G.case_names("ingest_dict_"))
def test_dict_snapshots_vs_reference(dev, case):
    meta, t = G.load(case)
    model = _model(meta, t, dev)
    seq = G.dict_sequence(meta, t, dev)
    for d in seq:
        d["x"] = d["x"].clone().requires_grad_(True)
    out = model(seq, labels=G.labels(meta, t, dev))
    G.assert_close("logits", out["logits"], t["out.logits"], OUT_ATOL, OUT_RTOL)
    G.assert_close("loss", out["loss"].reshape(1), t["out.loss"], OUT_ATOL, OUT_RTOL)
    out["loss"].backward()
    want = G.grads(t)
    for name, p in model.named_parameters():
        if name in want:
            G.assert_close("grad " + name, p.grad, want[name], GRAD_ATOL, GRAD_RTOL)
        else:
            assert p.grad is None, name
    for i, d in enumerate(seq):
        G.assert_close("grad x.%d" % i, d["x"].grad, t["grad.x.%d" % i], GRAD_ATOL, GRAD_RTOL)


@pytest.mark.parametrize("case", G.case_names("ingest_dict_"))
def test_snapshot_batch_matches_list(dev, case):
    """Host dicts -> SnapshotBatch (pinned, one H2D copy per array) gives bitwise the list path's outputs."""
    from tagan_amd.ingest import SnapshotBatch
    meta, t = G.load(case)
    model = _model(meta, t, dev)
    labels = G.labels(meta, t, dev)
    out1, g1 = _run(model, G.dict_sequence(meta, t, dev), labels)
    batch = model.ingest(G.dict_sequence(meta, t, "cpu"))
    assert isinstance(batch, SnapshotBatch) and batch.x.is_cuda and batch.node_counts == meta["n_list"]
    out2, g2 = _run(model, batch, labels)
    assert torch.equal(out1["logits"], out2["logits"]) and torch.equal(out1["loss"], out2["loss"])
    assert g1.keys() == g2.keys()
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    G.assert_close("batch logits", out2["logits"], t["out.logits"], OUT_ATOL, OUT_RTOL)


def test_global_index_on_device(dev):
    from tagan_amd.ingest import SnapshotBatch
    meta, t = G.load("ingest_dict_social")
    seq = G.dict_sequence(meta, t, "cpu")
    b_dev = SnapshotBatch.from_sequence(seq, dev)
    b_cpu = SnapshotBatch.from_sequence(seq, "cpu")
    u_d, i_d = b_dev.global_index()
    u_c, i_c = b_cpu.global_index()
    assert u_d.is_cuda and torch.equal(u_d.cpu(), u_c) and torch.equal(i_d.cpu(), i_c)


@pytest.mark.parametrize("packed", [False, True])
def test_out_of_range_edge_raises(dev, packed):
    """The reference's adj[edge_index[0], edge_index[1]] = 1 raises IndexError; so does the deferred check."""
    meta, t = G.load("ingest_dict_social")
    model = _model(meta, t, dev)
    seq = G.dict_sequence(meta, t, dev)
    n = int(seq[2]["x"].shape[0])
    seq[2]["edge_index"] = seq[2]["edge_index"].clone()
    seq[2]["edge_index"][1, 3] = n   # one past the last node of snapshot 2
    with pytest.raises(IndexError):
        model(model.ingest(seq) if packed else seq, labels=G.labels(meta, t, dev))
    torch.cuda.synchronize()
    out = model(G.dict_sequence(meta, t, dev), labels=G.labels(meta, t, dev))   # the model is still usable
    G.assert_close("logits after error", out["logits"], t["out.logits"], OUT_ATOL, OUT_RTOL)
