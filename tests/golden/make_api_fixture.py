"""Mint tests/golden/reference_layer_api.json: the constructor / forward signatures of the reference classes that
INTEGRATION.md §3's layer-level switch replaces, and the names the reference model.py imports from those modules.
Parses the reference with `ast` (nothing is imported or executed); run in the build container, where the reference
sits read-only at /root/reference:  python tests/golden/make_api_fixture.py"""
import ast
import json
import os

REF = "/root/reference/src/tagan"
MODULES = {   # module (relative to src/tagan) -> classes the switch serves
    "layers/geometric_attention.py": ["GeometricAttention", "DistanceMetric"],
    "layers/graph_attention.py": ["TAGANGraphAttention"],
    "layers/temporal_attention.py": ["TemporalAttention", "AsymmetricTemporalAttention", "TimeEncoding"],
    "utils/memory_bank.py": ["NodeMemoryBank"],
}


def _sig(fn):
    a = fn.args
    names = [x.arg for x in a.posonlyargs + a.args]
    defaults = [None] * (len(names) - len(a.defaults)) + [ast.unparse(d) for d in a.defaults]
    params = [{"name": n, "default": d} for n, d in zip(names, defaults)]
    params += [{"name": x.arg, "default": ast.unparse(d) if d is not None else None, "kwonly": True}
               for x, d in zip(a.kwonlyargs, a.kw_defaults)]
    if a.vararg:
        params.append({"name": "*" + a.vararg.arg, "default": None})
    if a.kwarg:
        params.append({"name": "**" + a.kwarg.arg, "default": None})
    return params


def main():
    out = {"note": "signatures parsed from the reference with ast (tests/golden/make_api_fixture.py)",
           "classes": {}, "model_imports": {}}
    for rel, classes in MODULES.items():
        tree = ast.parse(open(os.path.join(REF, rel)).read())
        for node in tree.body:
            if isinstance(node, ast.ClassDef) and node.name in classes:
                methods = {f.name: f for f in node.body if isinstance(f, ast.FunctionDef)}
                out["classes"][node.name] = {
                    "module": rel,
                    "bases": [ast.unparse(b) for b in node.bases],
                    "__init__": _sig(methods["__init__"]) if "__init__" in methods else None,
                    "forward": _sig(methods["forward"]) if "forward" in methods else None,
                    "public_methods": sorted(n for n in methods if not n.startswith("_")),
                }
    tree = ast.parse(open(os.path.join(REF, "model.py")).read())
    for node in tree.body:
        if isinstance(node, ast.ImportFrom) and node.module and node.level == 1:
            out["model_imports"].setdefault(node.module, sorted({a.name for a in node.names}))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_layer_api.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
