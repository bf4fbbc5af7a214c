"""tgn._cat_rows: the three sides' subgraph tensors concatenated along dim 0 -- a view when they are
consecutive row blocks of one tensor (a gathered pack), torch.cat otherwise -- equals torch.cat bit for
bit in every case, and prepare_contrast's conversions commute with it."""
import torch

from tempme_amd.tgn import _cat_rows


def test_adjacent_blocks_become_a_view():
    base = torch.arange(3 * 5 * 4, dtype=torch.int32).reshape(3, 5, 4)
    xs = list(base.unbind(0))
    out = _cat_rows(xs)
    assert torch.equal(out, torch.cat(xs))
    assert out.untyped_storage().data_ptr() == base.untyped_storage().data_ptr()   # no copy
    f = torch.rand(3, 5, 6)
    ys = [f[k] for k in range(3)]
    assert torch.equal(_cat_rows(ys).to(torch.float64), torch.cat([y.to(torch.float64) for y in ys]))


def test_other_layouts_are_copied():
    base = torch.arange(3 * 5 * 4, dtype=torch.int32).reshape(3, 5, 4)
    cases = [
        [base[0], base[2], base[1]],                          # out of order
        [base[0], base[1]],                                    # a prefix is still adjacent
        [base[:, :2][k] for k in range(3)],                    # non-contiguous slices
        [torch.zeros(5, 4, dtype=torch.int32) for _ in range(3)],   # separate storages
        [base[0], base[1].to(torch.int64), base[2]],           # mixed dtypes (torch.cat promotes)
    ]
    for xs in cases:
        assert torch.equal(_cat_rows(xs), torch.cat(xs))
    g = torch.rand(3, 5, 4, requires_grad=True)
    ys = list(g.unbind(0))
    out = _cat_rows(ys)
    assert out.grad_fn is not None and torch.equal(out, torch.cat(ys))


def test_single_row_blocks_with_odd_leading_stride():
    """B == 1: a [1, N] block is contiguous whatever its leading stride (is_contiguous ignores size-1 dims);
    the view must still lay the blocks out as consecutive rows, like torch.cat."""
    base = torch.arange(3 * 7, dtype=torch.int32).reshape(3, 7)
    xs = [base[k].as_strided((1, 7), (99, 1), base[k].storage_offset()) for k in range(3)]
    assert all(x.is_contiguous() for x in xs)
    out = _cat_rows(xs)
    assert torch.equal(out, torch.cat(xs))
    assert out.stride() == (7, 1)
