"""Loader for the committed golden fixtures in tests/golden/ (data only, no code)."""
import glob
import json
import os

import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names(prefix=""):
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.json")))


def load(case):
    with open(os.path.join(GOLDEN, case + ".json")) as f:
        meta = json.load(f)
    t = torch.load(os.path.join(GOLDEN, case + ".pt"), weights_only=True, map_location="cpu")
    return meta, t


def state_dict(t):
    return {k[3:]: v for k, v in t.items() if k.startswith("sd.")}


def grads(t):
    return {k[5:]: v for k, v in t.items() if k.startswith("grad.") and not k.startswith("grad.x")}


def sequence(meta, t, device="cpu"):
    seq = []
    for i in range(meta["T"]):
        x = t["in.x.%d" % i].to(device)
        ei = t["in.edge_index.%d" % i].to(device)
        ea = t.get("in.edge_attr.%d" % i)
        ea = ea.to(device) if ea is not None else None
        ids = t["in.node_ids.%d" % i].tolist()
        seq.append((x, ei, ea, ids))
    return seq


def dict_sequence(meta, t, device="cpu"):
    """The reference's snapshot dicts of an ingest_dict_* case (model.py:187-230): edge_attr only when stored."""
    seq = []
    for i in range(meta["T"]):
        d = {"x": t["in.x.%d" % i].to(device), "edge_index": t["in.edge_index.%d" % i].to(device),
             "node_ids": t["in.node_ids.%d" % i].tolist(), "timestep": float(t["in.timestep"][i])}
        if ("in.edge_attr.%d" % i) in t:
            d["edge_attr"] = t["in.edge_attr.%d" % i].to(device)
        seq.append(d)
    return seq


def labels(meta, t, device="cpu"):
    lab = t.get("in.labels")
    return lab.to(device) if lab is not None else None


# Observed errors of every assert_close, keyed by test id (written by conftest.py to $TAGAN_PARITY_LOG at the
# end of the session): {test: {check: [max_abs, max_rel_where_|want|>atol, normwise_rel, atol, rtol]}}.
ERRORS = {}


def _record(name, diff, want, atol, rtol):
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    finite = torch.isfinite(diff)
    d = diff[finite]
    w = want.abs()[finite]
    big = w > atol
    max_rel = float((d[big] / w[big]).max()) if bool(big.any()) else 0.0
    wn = float(w.norm())
    norm_rel = float(d.norm()) / wn if wn > 0 else float(d.norm())
    ERRORS.setdefault(test, {})[name] = [float(d.max()) if d.numel() else 0.0, max_rel, norm_rel, atol, rtol]


def normwise_rel(got, want):
    got = got.detach().to("cpu", torch.float64)
    want = want.detach().to("cpu", torch.float64)
    return float((got - want).norm()) / max(float(want.norm()), 1e-300)


def assert_close(name, got, want, atol, rtol=0.0):
    got = got.detach().to("cpu", torch.float64)
    want = want.detach().to("cpu", torch.float64)
    assert got.shape == want.shape, "%s: shape %s vs %s" % (name, tuple(got.shape), tuple(want.shape))
    both_nan = torch.isnan(got) & torch.isnan(want)
    diff = torch.where(both_nan, torch.zeros_like(got), (got - want).abs())
    _record(name, diff, want, atol, rtol)
    tol = atol + rtol * want.abs()
    bad = ~(diff <= torch.where(both_nan, torch.ones_like(tol), tol))
    if bad.any():
        i = int(bad.flatten().nonzero()[0])
        raise AssertionError("%s: max |diff| %.3e (atol %.1e rtol %.1e); first bad flat[%d] got %r want %r"
                             % (name, float(diff[~both_nan].max()), atol, rtol, i,
                                float(got.flatten()[i]), float(want.flatten()[i])))
