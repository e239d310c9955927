"""CPU checks of the C-ABI library: it loads without a GPU, exports every symbol of
include/tagan_hip.h, and its host-side helpers / argument validation behave."""
import ctypes

import numpy as np
import pytest
import torch

import tagan_amd
from tagan_amd import _lib


def test_library_loads_and_exports_header_symbols():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 12
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.tagan_version() >= 1


def _lowbias32(x):
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846CA68B)
        x = x ^ (x >> np.uint32(16))
    return x


def _drop_uniform(seed, stream, counter):
    """numpy restatement of tagan::drop_u(drop_key(seed, stream), counter) (common.cuh), used to
    regenerate dropout masks in tests; stream and counter broadcast against each other."""
    seed = int(seed)
    stream = np.asarray(stream, dtype=np.uint64)
    k = _lowbias32(np.uint32(seed & 0xFFFFFFFF) ^ np.uint32(0x9E3779B9))
    k = _lowbias32(k ^ np.uint32(seed >> 32))
    k = _lowbias32(k ^ (stream & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    k = _lowbias32(k ^ (stream >> np.uint64(32)).astype(np.uint32))
    u = _lowbias32(np.asarray(counter, dtype=np.uint32) ^ k) >> np.uint32(8)
    return u.astype(np.float64) / 16777216.0


def _drop_key(seed, stream):
    seed = int(seed)
    stream = np.asarray(stream, dtype=np.uint64)
    k = _lowbias32(np.uint32(seed & 0xFFFFFFFF) ^ np.uint32(0x9E3779B9))
    k = _lowbias32(k ^ np.uint32(seed >> 32))
    k = _lowbias32(k ^ (stream & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    return _lowbias32(k ^ (stream >> np.uint64(32)).astype(np.uint32))


def _temporal_keep(seed, stream, counter, p):
    """numpy restatement of the temporal attention dropout (temporal_attn.hip tkeep / include/tagan_hip.h): one
    lowbias32((c >> 1) ^ key) per counter pair, low half for the even counter, high half for the odd one, kept iff
    half >= ceil(p 2^16).  stream and counter broadcast against each other."""
    c = np.asarray(counter, dtype=np.uint32)
    w = _lowbias32((c >> np.uint32(1)) ^ _drop_key(seed, stream))
    half = np.where((c & np.uint32(1)) != 0, w >> np.uint32(16), w & np.uint32(0xFFFF))
    return half >= np.uint32(np.ceil(np.float32(p) * np.float32(65536.0)))


def test_temporal_dropout_statistics():
    """Keep rate of the pair-word temporal dropout at p = 0.1 / 0.5, and no correlation between the two halves of one
    word (even / odd counters) or between neighbouring pairs."""
    for p in (0.1, 0.5):
        k = _temporal_keep(7, np.arange(256, dtype=np.uint64)[:, None], np.arange(4096, dtype=np.uint32)[None, :], p)
        rate = k.mean()
        assert abs(rate - (1 - p)) < 4 * np.sqrt(p * (1 - p) / k.size), rate
        x = k.astype(np.float64)
        for a, b in ((x[:, 0::2], x[:, 1::2]), (x[:, 0:-2:2], x[:, 2::2])):
            r = np.corrcoef(a.ravel(), b.ravel())[0, 1]
            assert abs(r) < 4 / np.sqrt(a.size), r


def test_uniform_matches_numpy_restatement():
    L = _lib.lib()
    for seed in (0, 1, 123456789, 2 ** 62 - 1, 2 ** 64 - 1):
        for stream in (0, 7, 2 ** 33 + 5):
            ctr = np.array([0, 1, 2, 1000, 2 ** 31 + 3, 2 ** 32 - 1], dtype=np.uint32)
            want = _drop_uniform(seed, stream, ctr)
            got = np.array([L.tagan_uniform(seed, stream, int(c)) for c in ctr])
            np.testing.assert_array_equal(got.astype(np.float32), want.astype(np.float32))
            assert ((got >= 0) & (got < 1)).all()


def test_uniform_statistics():
    """Keep-rate and independence of the mask bits across streams / counters (p = 0.1)."""
    u = _drop_uniform(42, np.arange(64, dtype=np.uint64)[:, None], np.arange(20000, dtype=np.uint32)[None, :])
    keep = u >= 0.1
    assert abs(keep.mean() - 0.9) < 2e-3
    assert abs(u.mean() - 0.5) < 2e-3
    c = np.corrcoef(u[:8].reshape(8, -1))
    assert np.abs(c - np.eye(8)).max() < 0.03


def test_workspace_queries_are_host_only():
    L = _lib.lib()
    g = _lib.TaganGraph()
    g.n_nodes, g.chunk = 1000, 128
    g.chunk_cap = L.tagan_chunk_capacity(1000, 12000, 128)
    g.part_cap = L.tagan_part_capacity(12000, 128)
    assert g.chunk_cap == 1000 + 12000 // 128 + 1 and g.part_cap == 2 * (12000 // 128) + 2
    assert L.tagan_geo_attn_bwd_workspace(ctypes.byref(g), 8, 16) >= 1000 * 8 * 4
    assert L.tagan_geo_attn_fwd_workspace(ctypes.byref(g), 8, 16) >= g.part_cap * (16 + 128) * 4
    assert L.tagan_temporal_attn_bwd_workspace(100, 32, 8, 16) >= 100 * 8 * 63 * 4 + 100 * 3 * 128 * 4
    g.n_nodes = 0
    assert L.tagan_geo_attn_bwd_workspace(ctypes.byref(g), 8, 16) == 0


def test_argument_validation_reports_errors():
    L = _lib.lib()
    g = _lib.TaganGraph()
    rc = L.tagan_geo_attn_fwd(0, 99, ctypes.byref(g), 4, 16, None, None, None, 64, None, 0.0, 0, None, None, None,
                              None, 0, None)
    assert rc == -2
    assert b"metric" in L.tagan_last_error()
    rc = L.tagan_geo_attn_fwd(0, 0, ctypes.byref(g), 4, 16, None, None, None, 64, None, 0.0, 0, None, None, None,
                              None, 0, None)
    assert rc == -1 and b"graph" in L.tagan_last_error()
    rc = L.tagan_chunk_order(None, 10, None, None, None, 300, 12, None, None)
    assert rc == -1 and b"chunk_order" in L.tagan_last_error()
    rc = L.tagan_temporal_attn_fwd(7, 10, 4, 2, 8, None, None, None, 0, 0, None, None, 0, None, 0, 0, 0, 0.0, 0,
                                   None, 0, 0, None, None, None)
    assert rc == -2
    g.n_nodes, g.rowptr, g.col = 10, 16, 16   # non-null dummies: validation fails before any launch
    rc = L.tagan_geo_attn_fwd(0, 0, ctypes.byref(g), 4, 16, None, None, None, 64, None, 1.5, 0, None, None, None,
                              None, 0, None)
    assert rc == -1 and b"p_drop" in L.tagan_last_error()
    # the head kernels read x0, W1 and Wc1 as float4 runs: a pointer off 16 bytes is refused before any launch
    a, odd = 0x10000, 0x10004
    for W1 in (odd, a):
        x0 = a if W1 == odd else odd
        rc = L.tagan_head_fwd(1, 32, 128, 1, x0, W1, a, a, a, a, a, a, 1e-5, a, a, 0.0, 0, None, 0, a, a, None, a, None)
        assert rc == -1 and b"16-byte aligned" in L.tagan_last_error()


def test_no_cpu_path():
    from tagan_amd.kernels import GeoAttnFn, SnapshotGraph
    x = torch.zeros(4, 12)
    with pytest.raises(RuntimeError, match="HIP device"):
        GeoAttnFn.apply(x, None, None, 0, 1, 0.0, 0)


def test_metric_table_matches_header():
    with open(_lib.HEADER_PATH) as f:
        src = f.read()
    for name, mid in _lib.METRIC_IDS.items():
        assert ("TAGAN_METRIC_%s = %d" % (name.upper(), mid)) in src


def test_every_header_symbol_has_a_ctypes_signature():
    """A missing argtypes entry turns float arguments into ctypes errors at call time."""
    missing = [s for s in _lib.header_symbols() if s not in _lib._SIGNATURES]
    assert not missing, missing


def test_ctypes_signatures_match_header_arity():
    """Every ctypes signature has as many arguments as its declaration in include/tagan_hip.h (a miscounted
    argtypes list only fails at call time, on the GPU)."""
    import re
    with open(_lib.HEADER_PATH) as f:
        src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    bad = []
    for name, (_res, args) in _lib._SIGNATURES.items():
        m = re.search(r"\b%s\s*\(([^;{]*?)\)\s*;" % re.escape(name), src)
        assert m, "no declaration of %s" % name
        params = m.group(1).strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        if n != len(args):
            bad.append((name, n, len(args)))
    assert not bad, bad
