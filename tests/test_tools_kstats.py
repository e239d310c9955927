"""tools/kstats.py's kernel families: every kernel csrc/csr_build.hip defines is counted as "csr" (rounds 4-5
reported the C2 CSR build at 0.27 device-ms per step because the CSC-finish, partition and refine kernels fell into
"other"; the real figure was 0.49)."""
import csv
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CSR_SRC = os.path.join(ROOT, "temporal-asymmetric-graph-attention-network_amd", "csrc", "csr_build.hip")
PROFILE = os.path.join(ROOT, "profiles", "r5zk_c2_kernel_stats.csv")


def family(name):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kstats import FAMILIES
    return next((f for f, p in FAMILIES if re.search(p, name)), "other")


@pytest.fixture(autouse=True)
def _inputs():
    if not (os.path.exists(PROFILE) and os.path.exists(CSR_SRC)):
        pytest.skip("profile or source not in this tree")


def test_every_csr_builder_kernel_is_counted_as_csr():
    src = open(CSR_SRC).read()
    kernels = set(re.findall(r"__global__\s+void\s+(?:__launch_bounds__\([^)]*\)\s+)?(k_\w+)\s*\(", src))
    assert len(kernels) >= 10, kernels
    rows = list(csv.DictReader(open(PROFILE)))
    seen = 0
    for r in rows:
        m = re.search(r"\b(k_\w+)[<(]", r["Name"])
        if m and m.group(1) in kernels:
            seen += 1
            assert family(r["Name"]) == "csr", r["Name"]
    assert seen >= 8, seen


def test_edge_and_gemm_kernels_keep_their_families():
    rows = list(csv.DictReader(open(PROFILE)))
    for r in rows:
        n = r["Name"]
        if "k_geo_" in n:
            assert family(n) == "geo", n
        if "k_sgemm_nt" in n or "k_rowgemm" in n:
            assert family(n) == "sgemm (hand-written)", n
