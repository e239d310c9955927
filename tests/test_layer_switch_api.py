"""INTEGRATION.md §3's layer-level switch (the reference model.py kept, its layer modules replaced through
sys.modules) needs our modules to serve the same names with the same constructor / forward signatures.  Checked
against tests/golden/reference_layer_api.json (the reference's signatures parsed with ast by
tests/golden/make_api_fixture.py; the reference itself is not read here).  CPU only."""
import importlib
import inspect
import json
import os

import pytest

OURS = {   # reference module -> ours
    "layers/geometric_attention.py": "tagan_amd.layers.geometric_attention",
    "layers/graph_attention.py": "tagan_amd.layers.graph_attention",
    "layers/temporal_attention.py": "tagan_amd.layers.temporal_attention",
    "utils/memory_bank.py": "tagan_amd.utils.memory_bank",
}

with open(os.path.join(os.path.dirname(__file__), "golden", "reference_layer_api.json")) as f:
    API = json.load(f)


def _params(fn):
    out = []
    for p in inspect.signature(fn).parameters.values():
        name = ("*" if p.kind is p.VAR_POSITIONAL else "**" if p.kind is p.VAR_KEYWORD else "") + p.name
        out.append((name, None if p.default is p.empty else repr(p.default)))
    return out


def _ref_params(sig):
    return [(p["name"], p["default"]) for p in sig]


def _same_default(ours, ref):
    if ours is None or ref is None:
        return ours is None and ref is None
    try:   # the fixture holds source text ('0.1', "'euclidean'", 'None'): compare values where both are literals
        import ast
        return ast.literal_eval(ref) == ast.literal_eval(ours)
    except (ValueError, SyntaxError):
        return ours == ref


@pytest.mark.parametrize("cls", sorted(API["classes"]))
def test_class_signatures_match_reference(cls):
    spec = API["classes"][cls]
    mod = importlib.import_module(OURS[spec["module"]])
    ours = getattr(mod, cls, None)
    assert ours is not None, "%s missing from %s" % (cls, mod.__name__)
    for meth in ("__init__", "forward"):
        if spec[meth] is None:
            continue
        got, want = _params(getattr(ours, meth)), _ref_params(spec[meth])
        assert [n for n, _ in got] == [n for n, _ in want], "%s.%s parameters %s vs reference %s" % (
            cls, meth, [n for n, _ in got], [n for n, _ in want])
        for (n, d), (_, rd) in zip(got, want):
            assert _same_default(d, rd), "%s.%s(%s=...): default %s vs reference %s" % (cls, meth, n, d, rd)
    missing = [m for m in spec["public_methods"] if not hasattr(ours, m)]
    assert not missing, "%s lacks %s" % (cls, missing)


def test_model_imports_resolve():
    """Every name the reference model.py imports from a switched module exists in ours."""
    rel = {"layers.geometric_attention": "layers/geometric_attention.py", "layers.graph_attention":
           "layers/graph_attention.py", "layers.temporal_attention": "layers/temporal_attention.py"}
    for module, names in API["model_imports"].items():
        if module not in rel:
            continue   # the modules the switch leaves to the reference
        mod = importlib.import_module(OURS[rel[module]])
        for n in names:
            assert hasattr(mod, n), "%s.%s" % (mod.__name__, n)
