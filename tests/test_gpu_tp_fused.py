"""Fused backward of the interaction's output linear + TP (``eelg_tp_bwd_fused``) against the
unfused HIP path (the linear's grad-x kernel, then ``eelg_tp_bwd``), which the oracle tests pin
(``test_gpu_parity.py::test_interaction_block_fwd_bwd`` and the model-level tests run the fused
path by default against the fp64 oracle).

Tolerances: fp32 storage 1e-5 of each tensor's largest entry (both paths sum in fp32, in
different orders: MFMA vs the linear kernel for grad_agg); bf16 storage of grad_w / the per-edge
grad-x rows 1e-2 (one bf16 rounding, 2^-8 relative, of values whose fp32 sums differ in order).
"""
import pytest
import torch

from helpers import params

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _graph(n, e, seed, isolated=0):
    """random edges; the first ``isolated`` nodes receive none (zero-degree receivers)"""
    g = torch.Generator().manual_seed(seed)
    snd = torch.randint(0, n, (e,), generator=g)
    rcv = torch.randint(isolated, n, (e,), generator=g) if n > isolated else torch.zeros(0, dtype=torch.long)
    return torch.stack([snd, rcv[: snd.shape[0]]])


def _run(block, x, sh, ef, ei, go, fused):
    from gnn import ops
    old = ops.TP_BWF
    ops.TP_BWF = fused
    try:
        for p in block.parameters():
            p.grad = None
        xd = x.clone().requires_grad_(True)
        y, _ = block(xd, sh, ef, ei)
        (y * go).sum().backward()
        torch.cuda.synchronize()
        return y.detach(), xd.grad, {k: p.grad.clone() for k, p in block.named_parameters()}
    finally:
        ops.TP_BWF = old


@pytest.mark.parametrize("lmax,layer,n,e,isolated,storage", [
    (4, 1, 50, 200, 3, "float32"),
    (4, 1, 13, 40, 5, "float32"),        # one partial tile
    (4, 1, 5, 9, 0, "float32"),          # fewer receivers than a tile
    (4, 1, 3000, 12000, 17, "float32"),  # many tiles, XCD rounding of the grid
    (4, 0, 300, 1200, 2, "float32"),     # layer 0 (tpA: one input block)
    (3, 1, 777, 3100, 9, "float32"),
    (2, 1, 64, 256, 1, "float32"),
    (3, 1, 777, 3100, 9, "bfloat16"),    # BASELINE config 5 storage
    (4, 1, 300, 1200, 4, "bfloat16"),
])
def test_fused_linear_tp_backward_matches_unfused(lmax, layer, n, e, isolated, storage):
    from gnn.model import EnergyEquivGNN
    torch.manual_seed(0)
    m = EnergyEquivGNN(params(2, lmax=lmax, storage_dtype=storage)).to(DEV)
    blk = m.stiffness_head.layers[layer].interaction
    idx, _ = blk._config()
    assert blk._bwf(idx), "fused path not generated / not matching the linear"
    ei = _graph(n, e, 7 + n, isolated).to(DEV)
    din = blk.irreps_in.dim
    x = torch.randn(n, din, device=DEV)
    nsh = (lmax + 1) ** 2
    sh = torch.randn(e, nsh, device=DEV)
    ef = torch.rand(e, 12, device=DEV)
    go = torch.randn(n, blk.irreps_out.dim, device=DEV)
    y_ref, gx_ref, gp_ref = _run(blk, x, sh, ef, ei, go, False)
    y, gx, gp = _run(blk, x, sh, ef, ei, go, True)
    tol = 1e-5 if storage == "float32" else 1e-2
    assert torch.equal(y, y_ref)                       # same forward kernels
    assert rel_err(gx, gx_ref) < tol
    for k in gp_ref:
        # weight / bias gradients of the output linear come from the same kernels: bitwise
        if k.startswith("linear."):
            assert torch.equal(gp[k], gp_ref[k]), k
        else:
            assert rel_err(gp[k], gp_ref[k]) < tol, k


def test_fused_table_rejects_other_linears():
    """a linear whose layout is not the TP's merged-l3 one is refused (the unfused path runs)"""
    from gnn.model import EnergyEquivGNN
    from gnn.o3 import Linear
    from gnn import ops
    m = EnergyEquivGNN(params(2)).to(DEV)
    blk = m.stiffness_head.layers[1].interaction
    idx, _ = blk._config()
    blk._bwf(idx)
    other = Linear(blk.irreps_mid, "64x0e+32x1o+32x2e+32x3o+32x4e")
    assert not ops.tp_linear_fusable(idx, other, blk._tp_paths)


def _run_chunked(block, x, sh, ef, ei, go, chunks):
    from gnn import ops
    old = ops.TP_BWC
    ops.TP_BWC = chunks
    try:
        return _run(block, x, sh, ef, ei, go, False)
    finally:
        ops.TP_BWC = old


@pytest.mark.parametrize("lmax,n,e,isolated,chunks,storage", [
    (4, 3000, 12000, 17, 8, "float32"),
    (4, 50, 200, 3, 3, "float32"),
    (4, 5, 9, 0, 8, "float32"),          # more chunks than receivers
    (3, 777, 3100, 9, 4, "bfloat16"),
])
def test_chunked_linear_tp_backward_is_bitwise_unfused(lmax, n, e, isolated, chunks, storage):
    """EELG_TP_BWC: the linear's grad-x and tp_bwd per receiver chunk run the same kernels on
    row / edge sub-ranges, so every gradient equals the one-pass result bit for bit"""
    from gnn.model import EnergyEquivGNN
    torch.manual_seed(0)
    m = EnergyEquivGNN(params(2, lmax=lmax, storage_dtype=storage)).to(DEV)
    blk = m.stiffness_head.layers[1].interaction
    ei = _graph(n, e, 11 + n, isolated).to(DEV)
    x = torch.randn(n, blk.irreps_in.dim, device=DEV)
    sh = torch.randn(e, (lmax + 1) ** 2, device=DEV)
    ef = torch.rand(e, 12, device=DEV)
    go = torch.randn(n, blk.irreps_out.dim, device=DEV)
    y_ref, gx_ref, gp_ref = _run(blk, x, sh, ef, ei, go, False)
    y, gx, gp = _run_chunked(blk, x, sh, ef, ei, go, chunks)
    assert torch.equal(y, y_ref)
    assert torch.equal(gx, gx_ref)
    for k in gp_ref:
        assert torch.equal(gp[k], gp_ref[k]), k
