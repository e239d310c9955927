"""Pin the CPU oracle (oracle/) to golden vectors minted from the reference itself.

CPU-only.  Every oracle function is checked here before any GPU parity test
trusts it (tests/golden/make_golden.py made the fixtures; SURVEY.md §8c G1–G5).
"""
import pytest
import torch

import golden_io as G
import oracle
from oracle.tagan_oracle import geometric_attention, temporal_attention

ATOL, RTOL = 2e-5, 2e-4


def _leaves(sd):
    return {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}


@pytest.mark.parametrize("case", G.case_names("e2e_"))
@pytest.mark.parametrize("mode", ["sparse", "dense"])
def test_e2e(case, mode):
    meta, t = G.load(case)
    if mode == "dense" and max(meta["n_list"]) > 100:
        pytest.skip("dense mode checked on the small cases")
    P = _leaves(G.state_dict(t))
    seq = G.sequence(meta, t)
    seq = [(x.clone().requires_grad_(True), ei, ea, ids) for x, ei, ea, ids in seq]
    lab = G.labels(meta, t)
    col = {}
    out = oracle.tagan_forward(P, meta["config"], seq, lab, meta.get("return_attention_weights", False),
                               mode=mode, collect=col)
    G.assert_close("logits", out["logits"], t["out.logits"], ATOL, RTOL)
    G.assert_close("predictions", out["predictions"], t["out.predictions"], ATOL, RTOL)
    if "out.graph_features" in t:
        G.assert_close("graph_features", col["graph_features"], t["out.graph_features"], ATOL, RTOL)
    if "out.temporal" in t:
        G.assert_close("temporal", col["temporal"], t["out.temporal"], ATOL, RTOL)
    for i in range(meta["T"]):
        if "out.geo.%d" % i in t:
            G.assert_close("geo.%d" % i, col["geo"][i], t["out.geo.%d" % i], ATOL, RTOL)
    if meta.get("return_attention_weights"):
        G.assert_close("tattn", out["temporal_attention_weights"], t["out.temporal_attention_weights"], ATOL, RTOL)
        assert len(out["geometric_attention_weights"]) == meta["n_geo_attn_weights"]
    if out["loss"] is None:
        assert "out.loss" not in t
        return
    G.assert_close("loss", out["loss"].reshape(1), t["out.loss"], ATOL, RTOL)
    out["loss"].backward()
    want = G.grads(t)
    for name, p in P.items():
        if name in want:
            assert p.grad is not None, name
            G.assert_close("grad " + name, p.grad, want[name], 5e-5, 1e-3)
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
    for i, (x, _, _, _) in enumerate(seq):
        G.assert_close("grad x.%d" % i, x.grad, t["grad.x.%d" % i], 5e-5, 1e-3)


@pytest.mark.parametrize("case", G.case_names("gat_"))
@pytest.mark.parametrize("mode", ["sparse", "dense", "dense_faithful"])
def test_graph_attention(case, mode):
    meta, t = G.load(case)
    P = _leaves(G.state_dict(t))
    P = {"g." + k: v for k, v in P.items()}
    x = t["in.x"].clone().requires_grad_(True)
    out = oracle.graph_attention(x, t["in.edge_index"], P, "g", meta["heads"], meta["metric"], True,
                                 meta["learnable_distance"], mode=mode)
    G.assert_close("out", out, t["out"], ATOL, RTOL)
    (out * t["in.grad_out"]).sum().backward()
    G.assert_close("grad x", x.grad, t["grad.x"], 5e-5, 1e-3)
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, P["g." + name].grad, g, 5e-5, 1e-3)


@pytest.mark.parametrize("case", G.case_names("geo_"))
@pytest.mark.parametrize("mode", ["sparse", "dense"])
def test_geometric_attention(case, mode):
    meta, t = G.load(case)
    P = {"m." + k: v for k, v in _leaves(G.state_dict(t)).items()}
    x = t["in.x"].clone().requires_grad_(True)
    out = geometric_attention(x, P, "m", meta["heads"], meta["metric"], True, False,
                              attention_mask=t.get("in.mask"), geometric_bias=t.get("in.bias"), mode=mode)
    G.assert_close("out", out, t["out"], ATOL, RTOL)
    (out * t["in.grad_out"]).sum().backward()
    G.assert_close("grad x", x.grad, t["grad.x"], 5e-5, 1e-3)
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, P["m." + name].grad, g, 5e-5, 1e-3)


@pytest.mark.parametrize("case", G.case_names("tatt_"))
def test_temporal_attention(case):
    meta, t = G.load(case)
    P = {"m." + k: v for k, v in _leaves(G.state_dict(t)).items()}
    ctor = meta["ctor"]
    if meta["x_kind"] == "list":
        xs = [t["in.x.%d" % i].clone().requires_grad_(True) for i in range(meta["T"])]
        x_in = xs
    else:
        xs = [t["in.x"].clone().requires_grad_(True)]
        x_in = xs[0]
    cls = "asym" if meta["cls"] == "AsymmetricTemporalAttention" else "base"
    kw = dict(cls=cls, causal=ctor.get("causal", False), use_layer_norm=ctor.get("use_layer_norm", True),
              relative_position_bias=ctor.get("relative_position_bias", True),
              max_relative_position=ctor.get("max_relative_position", 32),
              asymmetric_window_size=ctor.get("asymmetric_window_size", 5),
              time_aware=ctor.get("time_aware", True), use_time_masks=ctor.get("use_time_masks", True),
              time_stamps=t.get("in.time_stamps"), attention_mask=t.get("in.mask"),
              return_attention_weights=meta["with_attn"])
    res = temporal_attention(x_in, P, "m", meta["heads"], **kw)
    out, w = res if meta["with_attn"] else (res, None)
    G.assert_close("out", out, t["out"], ATOL, RTOL)
    if w is not None:
        G.assert_close("attn", w, t["out.attn"], ATOL, RTOL)
    (out * t["in.grad_out"]).sum().backward()
    for i, xi in enumerate(xs):
        key = "grad.x.%d" % i if meta["x_kind"] == "list" else "grad.x"
        G.assert_close(key, xi.grad, t[key], 5e-5, 1e-3)
    for name, g in G.grads(t).items():
        G.assert_close("grad " + name, P["m." + name].grad, g, 5e-5, 1e-3)


def test_membank_trace():
    meta, t = G.load("membank_trace")
    bank = oracle.NodeMemoryBankOracle(meta["H"], meta["decay_factor"], meta["max_inactivity"])
    for k, rec in enumerate(meta["ops"]):
        if rec["op"] == "update":
            bank.update(rec["ids"], t["op%d.states" % k], rec["t"])
        elif rec["op"] == "update_state":
            bank.update_state(rec["ids"][0], t["op%d.states" % k][0], rec["t"])
        elif rec["op"] == "get_states":
            G.assert_close("get_states", bank.get_states(rec["ids"]), t["op%d.result" % k], 1e-7)
        elif rec["op"] == "decay_all":
            bank.decay_all()
        assert sorted(bank.node_states) == rec["keys"], k
        assert {str(i): c for i, c in sorted(bank.inactivity_counter.items())} == rec["inactivity"], k
        assert {str(i): c for i, c in sorted(bank.last_seen.items())} == rec["last_seen"], k
        assert {str(i): c for i, c in sorted(bank.frequency.items())} == rec["frequency"], k
        assert bank.size == rec["size"], k
        if rec["keys"]:
            got = torch.stack([bank.node_states[i] for i in rec["keys"]])
            G.assert_close("states op%d" % k, got, t["op%d.bank_states" % k], 1e-6)


def test_csr_semantics():
    ei = torch.tensor([[0, 0, 1, 2, 2, -1], [1, 1, 1, 0, 2, 0]])
    rowptr, col = oracle.csr_from_edge_index(ei, 4)
    assert rowptr.tolist() == [0, 2, 3, 5, 7]
    assert col.tolist() == [0, 1, 1, 0, 2, 0, 3]
    with pytest.raises(IndexError):
        oracle.csr_from_edge_index(torch.tensor([[0], [4]]), 4)


def _tprop_run(meta, t, P, prop):
    """Run one tprop_* case through ``prop`` (oracle.tprop_oracle or the device module's functional form)."""
    kind, kw = meta["module"], dict(meta["ctor"])
    kw.pop("dropout", None)
    ts = t.get("in.time_stamps")
    if kind == "gating":
        cur = t["in.current"].clone().requires_grad_(True)
        prev = t["in.previous"].clone().requires_grad_(True)
        return [prop.gating_unit(cur, prev, P, "", **{k: v for k, v in kw.items() if k == "residual"})], [cur, prev]
    xs = [t["in.x.%d" % i].clone().requires_grad_(True) for i in range(meta["T"])]
    if kind == "evolution":
        outs = prop.evolution_layer(xs, ts, P, "", kw.get("time_aware", True), kw.get("bidirectional", False),
                                    kw.get("residual", True))
    elif kind == "skip":
        outs = prop.skip_connection(xs, P, "", kw.get("window_size", 3), kw.get("aggregation", "mean"),
                                    kw.get("residual", True))
    else:
        outs = prop.propagation(xs, ts, P, "", kw.get("time_aware", True), kw.get("bidirectional", False),
                                kw.get("use_skip_connection", True), kw.get("window_size", 3),
                                kw.get("aggregation", "mean"), kw.get("residual", True))
    return outs, xs


@pytest.mark.parametrize("case", G.case_names("tprop_"))
def test_temporal_propagation_intended(case):
    from oracle import tprop_oracle
    meta, t = G.load(case)
    sd = {k[3:].lstrip("."): v for k, v in t.items() if k.startswith("sd.")}
    P = _leaves(sd)
    # the oracle takes "<prefix>.<param>" names; with an empty prefix strip the leading dot it adds
    P = _DotKeys(P)
    outs, xs = _tprop_run(meta, t, P, tprop_oracle)
    for i, o in enumerate(outs):
        G.assert_close("out.%d" % i, o, t["out.%d" % i], ATOL, RTOL)
    sum((o * t["in.grad_out.%d" % i]).sum() for i, o in enumerate(outs)).backward()
    for i, x in enumerate(xs):
        G.assert_close("grad.x.%d" % i, x.grad, t["grad.x.%d" % i], ATOL, RTOL)
    for k, v in P.items():
        if "grad." + k in t:
            G.assert_close("grad." + k, v.grad, t["grad." + k], ATOL, RTOL)
        else:
            assert v.grad is None or not v.grad.any(), k


class _DotKeys(dict):
    """Parameter mapping that also answers ".name" for "name" (empty module prefix)."""

    def __getitem__(self, k):
        return super().__getitem__(k[1:] if k.startswith(".") else k)

    def __contains__(self, k):
        return super().__contains__(k[1:] if k.startswith(".") else k)

    def get(self, k, d=None):
        return self[k] if k in self else d
