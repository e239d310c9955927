"""INTEGRATION.md's C-ABI table names only entry points that include/tagan_hip.h declares (and the library exports).

A row names full symbols (`tagan_geo_attn_fwd`) and suffix shorthands of the row's first symbol (`_bwd`, `_fwd_keep`):
a shorthand resolves when replacing one to three trailing `_`-components of that symbol with it gives a declared name.
"""
import os
import re

from tagan_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table_rows():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 4. C-ABI"):]
    sec = sec[:sec.index("\n## ", 5)] if "\n## " in sec[5:] else sec
    return [ln for ln in sec.splitlines() if ln.startswith("| `tagan_")]


def _declared():
    hdr = open(os.path.join(ROOT, "include", "tagan_hip.h")).read()
    return set(re.findall(r"\b(tagan_[a-z0-9_]+)\s*\(", hdr))


def test_integration_table_names_are_declared():
    decl = _declared()
    rows = _table_rows()
    assert len(rows) >= 10
    bad = []
    for row in rows:
        cell = row.split("|")[1]
        toks = re.findall(r"`(_?tagan_[a-z0-9_]+|_[a-z0-9_]+)`", cell)
        full = [t for t in toks if t.startswith("tagan_")]
        assert full, row
        base = full[0]
        for t in toks:
            if t.startswith("tagan_"):
                if t not in decl:
                    bad.append(t)
                continue
            parts = base.split("_")
            cands = ["_".join(parts[:-k]) + t for k in (1, 2, 3) if len(parts) > k]
            if not any(c in decl for c in cands):
                bad.append(base + " ~ " + t)
    assert not bad, bad


def test_integration_table_names_are_exported():
    L = _lib.lib()
    for row in _table_rows():
        for t in re.findall(r"`(tagan_[a-z0-9_]+)`", row.split("|")[1]):
            assert hasattr(L, t), t
