"""Snapshot ingestion on the CPU: the oracle on the reference's snapshot DICTS against the goldens minted from
the reference itself (tests/golden/ingest_dict_*: global user ids, variable node counts, edge_attr absent or
present; model.py:187-230), the SnapshotBatch packing layout and its reference error behaviour, and the
social generator's stated shape (degree law, unique edges, global ids)."""
import pytest
import torch

import golden_io as G
from oracle import tagan_oracle as oracle

CASES = G.case_names("ingest_dict_")


def test_cases_present():
    assert CASES == ["ingest_dict_social", "ingest_dict_social_ea"]


@pytest.mark.parametrize("case", CASES)
def test_oracle_on_dict_snapshots(case):
    meta, t = G.load(case)
    assert meta["format"] == "dict"
    P = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in G.state_dict(t).items()}
    seq = G.dict_sequence(meta, t)
    assert all(("edge_attr" in d) == meta["with_edge_attr"] for d in seq)
    for d in seq:
        d["x"] = d["x"].clone().requires_grad_(True)
    out = oracle.tagan_forward(P, meta["config"], seq, G.labels(meta, t))
    G.assert_close("logits", out["logits"], t["out.logits"], 2e-5, 1e-4)
    G.assert_close("loss", out["loss"].reshape(1), t["out.loss"], 2e-5, 1e-4)
    out["loss"].backward()
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, P[name].grad, g, 5e-5, 1e-3)
    for i, d in enumerate(seq):
        G.assert_close("grad x.%d" % i, d["x"].grad, t["grad.x.%d" % i], 5e-5, 1e-3)


@pytest.mark.parametrize("case", CASES)
def test_snapshot_batch_layout(case):
    from tagan_amd.ingest import SnapshotBatch
    meta, t = G.load(case)
    seq = G.dict_sequence(meta, t)
    b = SnapshotBatch.from_sequence(seq, "cpu")
    assert b.node_counts == meta["n_list"] and b.num_snapshots == meta["T"]
    assert b.timesteps == [float(v) for v in t["in.timestep"]]
    assert (b.edge_attr is not None) == meta["with_edge_attr"]
    for i, d in enumerate(seq):
        x, ei, ea, ids = b.snapshot(i)
        assert torch.equal(x, d["x"]) and torch.equal(ei, d["edge_index"]) and ids == d["node_ids"]
        if meta["with_edge_attr"]:
            assert torch.equal(ea, d["edge_attr"])
    # the reference's sorted global id list and node_id_to_idx (model.py:184-201)
    all_ids = sorted(set(i for d in seq for i in d["node_ids"]))
    uniq, inv = b.global_index()
    assert uniq.tolist() == all_ids
    flat = [i for d in seq for i in d["node_ids"]]
    assert [all_ids[k] for k in inv.tolist()] == flat
    # tuple and dict forms pack identically
    b2 = SnapshotBatch.from_sequence([(d["x"], d["edge_index"], d.get("edge_attr"), d["node_ids"]) for d in seq],
                                     "cpu")
    assert torch.equal(b.x, b2.x) and torch.equal(b.edge_index, b2.edge_index) and b.edge_ptr == b2.edge_ptr


def test_snapshot_batch_errors():
    from tagan_amd.ingest import SnapshotBatch
    x, ei = torch.randn(5, 3), torch.zeros(2, 4, dtype=torch.int64)
    with pytest.raises(ValueError, match="Expected at least 4 elements"):
        SnapshotBatch.from_sequence([(x, ei, None)], "cpu")
    with pytest.raises(ValueError, match="Unsupported snapshot type"):
        SnapshotBatch.from_sequence([[x, ei, None, [0] * 5]], "cpu")
    with pytest.raises(KeyError):
        SnapshotBatch.from_sequence([{"x": x, "edge_index": ei}], "cpu")   # the reference's snapshot['node_ids']
    # the reference never checks one id per row (model.py:186-204): accepted, marked, snapshot() refuses
    b = SnapshotBatch.from_sequence([(x, ei, None, [0, 1])], "cpu")
    assert not b.ids_row_aligned and b.global_index()[0].tolist() == [0, 1]
    with pytest.raises(ValueError, match="node ids"):
        b.snapshot(0)


def test_snapshot_batch_string_ids():
    """Non-integer global ids (string user ids): coded by rank in sorted(set(ids)), the reference's
    all_node_ids order (model.py:184-201); snapshot() gives the original ids back."""
    from tagan_amd.ingest import SnapshotBatch
    g = torch.Generator().manual_seed(3)
    ids0, ids1 = ["u17", "u03", "u99"], ["u03", "alice", "u17", "bob"]
    seq = [(torch.randn(3, 4, generator=g), torch.tensor([[0, 1], [2, 0]]), None, ids0),
           (torch.randn(4, 4, generator=g), torch.tensor([[0, 3], [1, 2]]), None, ids1)]
    b = SnapshotBatch.from_sequence(seq, "cpu")
    all_ids = sorted(set(ids0 + ids1))
    assert b.id_values == all_ids and b.ids_row_aligned
    uniq, inv = b.global_index()
    assert [all_ids[k] for k in uniq.tolist()] == all_ids
    assert [all_ids[k] for k in inv.tolist()] == ids0 + ids1
    assert b.snapshot(0)[3] == ids0 and b.snapshot(1)[3] == ids1


def test_social_generator_shape():
    from tagan_amd.synthetic import make_social_snapshots, unique_edges
    seq = make_social_snapshots(6, 2000, 20000, seed=5)
    counts = [int(d["x"].shape[0]) for d in seq]
    assert len(set(counts)) > 1 and all(1200 <= n <= 1800 for n in counts)   # variable active users
    for d in seq:
        n = int(d["x"].shape[0])
        assert d["x"].shape[1] == 27 and d["edge_attr"].shape == (20000, 2)
        assert int(d["edge_index"].min()) >= 0 and int(d["edge_index"].max()) < n
        assert len(set(d["node_ids"])) == n and min(d["node_ids"]) >= 1000
        u = unique_edges(d["edge_index"], n)
        assert 0.3 * 20000 < u < 0.95 * 20000          # Zipf hubs repeat pairs: the set is smaller than E
        deg = torch.bincount(d["edge_index"][0], minlength=n).sort(descending=True).values.double()
        assert deg[0] > 20 * deg.mean()                  # power-law out-degree: a hub far above the mean
    assert sorted(set(i for d in seq for i in d["node_ids"])) != []
