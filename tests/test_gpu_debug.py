"""The bounds-check build (``make debug`` -> libtagan_hip_debug.so): a corrupted gather index or
partial slot is caught by the device checks, skipped, and reported by the launch check as TAGAN_ERR_LAUNCH naming the
failing source line -- instead of an out-of-bounds access.  The corrupt-input cases run ONLY on the debug build
(``TAGAN_LIB=.../libtagan_hip_debug.so``): on the shipped build the same inputs would be real out-of-bounds accesses."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(dev, n=300, e=2000, seed=3):
    from tagan_amd.kernels import build_graph
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=g).to(dev)
    return build_graph([ei], [n])


def _is_debug():
    from tagan_amd._lib import lib
    return bool(lib().tagan_debug_build())


def test_debug_flag_matches_library_name():
    from tagan_amd import _lib
    assert _is_debug() == _lib.LIB_PATH.endswith("_debug.so")


@pytest.mark.parametrize("what", ["col", "seg"])
def test_debug_build_catches_corrupt_graph(what):
    if not _is_debug():
        pytest.skip("corrupt-input cases need the bounds-check build (TAGAN_LIB=.../libtagan_hip_debug.so)")
    from tagan_amd.kernels import _geo_fwd
    dev = torch.device("cuda:0")
    graph = _graph(dev)
    n, heads, H = graph.num_nodes, 4, 64
    qkv = torch.randn(n, 3 * H, device=dev)
    out = torch.empty(n, H, device=dev)
    lse = torch.empty(n, heads, device=dev)
    _geo_fwd(qkv, graph, 0, heads, None, 0.0, 0, out, lse, None)    # clean graph: no check fires
    torch.cuda.synchronize()
    if what == "col":
        graph.col[5] = n + 7                  # a neighbour id past the node count (a gather index)
    else:
        graph.row_chunks[1][0] = n + 3        # a chunk's segment (row) past the node count
    with pytest.raises(RuntimeError, match="TAGAN_DEBUG check failed"):
        _geo_fwd(qkv, graph, 0, heads, None, 0.0, 0, out, lse, None)
    torch.cuda.synchronize()
