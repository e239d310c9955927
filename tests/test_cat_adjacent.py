"""kernels.cat_adjacent: a view when the pieces are back to back in one buffer, torch.cat otherwise (CPU)."""
import torch

from tagan_amd.kernels import cat_adjacent


def test_adjacent_columns_are_a_view():
    base = torch.arange(2 * 12).view(2, 12)
    parts = [base[:, 0:5], base[:, 5:5], base[:, 5:12]]
    out = cat_adjacent(parts, 1)
    assert torch.equal(out, torch.cat(parts, 1))
    assert out.data_ptr() == base.data_ptr() and out.stride() == base.stride()


def test_adjacent_rows_are_a_view():
    base = torch.randn(10, 3)
    parts = [base[0:4], base[4:9]]
    out = cat_adjacent(parts, 0)
    assert torch.equal(out, base[:9]) and out.data_ptr() == base.data_ptr()


def test_non_adjacent_falls_back_to_cat():
    base = torch.arange(20).view(2, 10)
    for parts, dim in (([base[:, 0:3], base[:, 4:6]], 1),                 # gap
                       ([base[:, 4:6], base[:, 0:4]], 1),                 # out of order
                       ([torch.zeros(2, 3, dtype=base.dtype), base[:, 3:5]], 1),   # other buffers
                       ([base[0:1, 0:3], base[:, 3:5]], 1)):              # other extent
        try:
            want = torch.cat(parts, dim)
        except RuntimeError:
            continue
        out = cat_adjacent(parts, dim)
        assert torch.equal(out, want)
        assert out.data_ptr() != base.data_ptr() or parts[0].data_ptr() != base.data_ptr()


def test_pieces_that_require_grad_get_their_gradients():
    """Adjacent views of one leaf that requires grad: every piece's rows get their gradient (torch.cat semantics; an
    as_strided view of the first piece would drop the others')."""
    leaf = torch.randn(10, 3, requires_grad=True)
    parts = [leaf[0:4], leaf[4:7], leaf[7:10]]
    w = torch.randn(10, 3)
    (cat_adjacent(parts, 0) * w).sum().backward()
    assert torch.equal(leaf.grad, w)
    with torch.no_grad():
        out = cat_adjacent([p.detach() for p in parts], 0)
    assert out.data_ptr() == leaf.data_ptr()
