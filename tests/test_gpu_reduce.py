"""``eelg_sum_rows``: the deterministic partial-sum / bias-gradient reduction against an fp64
sum, over one- and two-pass row counts, ragged and strided layouts, and a bitwise repeat."""
import pytest
import torch

DEV = "cuda"

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 7), (64, 5120), (94, 1344 * 64), (512, 4992),
                                       (256, 36), (257, 36), (40000, 32), (7, 240640), (2049, 3)])
def test_sum_rows_matches_fp64(rows, cols):
    from gnn import ops
    torch.manual_seed(rows + cols)
    part = torch.randn(rows, cols, device=DEV)
    out = ops.sum_rows(part)
    assert out.shape == (cols,)
    assert _rel(out, part.double().sum(0)) < 2e-6
    assert torch.equal(ops.sum_rows(part), out)          # fixed order: bitwise repeatable


def test_sum_rows_strided_column_block_and_shapes():
    """a column block of a wider row-major tensor (the bias gradient of one output slot), a
    misaligned block (scalar path), a 3-D partial buffer, scale, and zero rows"""
    from gnn import ops
    torch.manual_seed(3)
    g = torch.randn(32768, 800, device=DEV)
    for off, m in ((0, 32), (3, 29), (768, 32)):
        out = ops.sum_rows(g[:, off: off + m])
        assert _rel(out, g[:, off: off + m].double().sum(0)) < 2e-6
    p3 = torch.randn(64, 32, 7520, device=DEV)
    assert _rel(ops.sum_rows(p3, scale=0.5), 0.5 * p3.double().sum(0)) < 2e-6
    dst = torch.full((40,), float("nan"), device=DEV)
    ops.sum_rows(torch.randn(5, 8, device=DEV), out=dst[8:16])
    assert torch.isnan(dst[:8]).all() and torch.isnan(dst[16:]).all() and torch.isfinite(dst[8:16]).all()
    z = ops.sum_rows(torch.empty(0, 12, device=DEV))
    assert torch.equal(z, torch.zeros(12, device=DEV))
