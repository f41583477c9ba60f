"""BASELINE config 5: bf16 storage of the edge-sized interaction tensors, fp32 arithmetic.

Tolerances (stated per test):
* kernel level, bf16 kernel vs the fp32 kernel fed the same bf16-rounded weights: the forward
  reads identical values in identical order -> 1e-6; grad_w is the fp32 gradient rounded once
  to bf16 -> 2^-8 relative per element; grad_x sums bf16-rounded per-edge terms -> 1e-2;
* end to end vs the fp64 oracle (SURVEY.md section 8c, bf16 variant): stiffness and loss
  2e-2 relative; parameter gradients: all gradients together 2e-2 relative to their max, and
  every parameter's gradient at cosine similarity >= 0.999 with the oracle's (a per-parameter
  max-relative bound is meaningless for parameters whose gradient is ~1e-3 of the others',
  e.g. layer 0's 3o contraction weights, where bf16 noise of the large terms dominates).
"""
import pytest
import torch

from helpers import batch, batch_to, copy_params, params, record_parity

import oracle.model as omodel
from oracle.train import stiffness_loss as oracle_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("lmax,layer0", [(4, False), (4, True), (3, False)])
def test_tp_interaction_bf16_storage(lmax, layer0):
    from gnn import _lib, cg, ops
    from gnn.irreps import Irreps
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    csr = ops.EdgeCSR.build(bd.edge_index, b.node_attrs.shape[0])
    sh_ir = Irreps.spherical_harmonics(lmax)
    mul = 32
    node = Irreps(f"{mul}x0e") if layer0 else Irreps(
        "+".join(f"{mul}x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1)))
    target = (sh_ir * mul).sort()[0].simplify()
    idx, info = _lib.tp_config_by_sig(cg.fnv1a64(cg.tp_signature(node, sh_ir, target)))
    sh, _ = ops.edge_embed(bd.positions, csr, bd.shifts[csr.perm],
                           bd.edge_attr[csr.perm].reshape(-1), lmax, 6, 0.6, rmax)
    torch.manual_seed(5)
    n, e = csr.num_nodes, csr.num_edges
    x = torch.randn(n, info["din"], device=DEV)
    wb = torch.randn(e, info["wn"], device=DEV).to(torch.bfloat16)
    g = torch.randn(n, info["dmid"], device=DEV)

    def run(w):
        xx = x.clone().requires_grad_(True)
        ww = w.clone().requires_grad_(True)
        agg = ops.tp_interaction(xx, sh, ww, csr, idx, info, 0.25)
        (agg * g).sum().backward()
        return agg, xx.grad, ww.grad

    a16, gx16, gw16 = run(wb)
    a32, gx32, gw32 = run(wb.float())
    assert gw16.dtype == torch.bfloat16 and a16.dtype == torch.float32
    assert rel_err(a16, a32) < 1e-6
    # one rounding of each grad_w element to bf16 (relative 2^-9, bounded by 2^-8 here)
    gwr = (gw16.float() - gw32).abs() / gw32.abs().clamp_min(1e-30)
    assert float(gwr[gw32.abs() > 1e-6 * gw32.abs().max()].max()) < 2 ** -8
    assert rel_err(gx16, gx32) < 1e-2


def test_segment_sum_bf16_source():
    from gnn import ops
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    csr = ops.EdgeCSR.build(bd.edge_index, b.node_attrs.shape[0])
    for width in (800, 3):
        src = torch.randn(csr.num_edges, width, device=DEV).to(torch.bfloat16)
        out = ops.segment_sum_csr(src, csr.srowptr, csr.num_nodes, idx=csr.sperm)
        ref = torch.zeros(csr.num_nodes, width, dtype=torch.float64).index_add_(
            0, csr.sender.long().cpu(), src.double().cpu())
        assert out.dtype == torch.float32
        assert rel_err(out, ref) < 1e-6


@pytest.mark.parametrize("lmax", [3, 4])
def test_model_bf16_storage_matches_oracle(lmax):
    """lmax 3 = BASELINE config 5 (SH and hidden irreps up to l = 3, bf16 storage)."""
    from gnn.model import EnergyEquivGNN
    from gnn.train import stiffness_loss
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    p = params(2, lmax=lmax, max_edge_radius=rmax)
    torch.manual_seed(0)
    o = omodel.EnergyEquivGNN(p).double()
    p.storage_dtype = "bfloat16"
    m = EnergyEquivGNN(p).to(DEV)
    copy_params(o, m)
    bo = batch_to(b, "cpu", torch.float64)
    co = o(bo)["stiffness"]
    lo = oracle_loss(co, bo.stiffness)
    lo.backward()
    cm = m(bd)["stiffness"]
    lm = stiffness_loss(cm, bd.stiffness)
    lm.backward()
    assert rel_err(cm, co) < 2e-2
    assert abs(lm.item() - lo.item()) <= 2e-2 * abs(lo.item())
    po = dict(o.named_parameters())
    names = [n for n, _ in m.named_parameters()]
    gm = torch.cat([pm.grad.double().cpu().reshape(-1) for _, pm in m.named_parameters()])
    go = torch.cat([po[n].grad.reshape(-1) for n in names])
    assert rel_err(gm, go) < 2e-2
    cos_min = 1.0
    for name, pm in m.named_parameters():
        a, r = pm.grad.double().cpu().reshape(-1), po[name].grad.reshape(-1)
        if float(r.norm()) == 0.0:          # structurally unused output (e.g. the last layer's 1o)
            assert float(a.abs().max()) <= 1e-6 * float(go.abs().max()), name
            continue
        cos = float(a @ r / (a.norm() * r.norm()).clamp_min(1e-300))
        cos_min = min(cos_min, cos)
        assert cos >= 0.999, (name, cos)
    record_parity(f"bf16_model_l{lmax}", stiffness=rel_err(cm, co),
                  grad_all=rel_err(gm, go), cos_min=cos_min)


@pytest.mark.parametrize("lmax,layer0,bf,mul", [(4, False, False, 32), (4, True, False, 32), (3, False, False, 32),
                                                (4, False, True, 32), (3, False, True, 32),
                                                (4, False, False, 16), (4, False, False, 64), (2, True, False, 64)])
def test_tp_bwd_sender_order_matches_edge_order(lmax, layer0, bf, mul):
    """eelg_tp_bwd_sender (grad_x summed per sender in registers) vs eelg_tp_bwd + the sender
    segment sum, on a graph whose first 7 nodes send nothing (their grad_x must be 0).
    grad_w: the same per-edge expression (fma contraction may differ) -> 1e-6 fp32, one
    bf16 ulp (2^-8) with bf16 storage; grad_x fp32: same order, fma vs add
    -> 1e-6; bf16 storage: the edge path rounds each per-edge term to bf16 -> 1e-2."""
    from gnn import _lib, cg, ops
    from gnn.irreps import Irreps
    b, rmax = batch(4, 50, 200, 1234)
    keep = b.edge_index[0] >= 7                       # nodes 0..6 have no out-edges
    ei = b.edge_index[:, keep]
    bd = b.to(DEV)
    csr = ops.EdgeCSR.build(ei.to(DEV), b.node_attrs.shape[0])
    sh_ir = Irreps.spherical_harmonics(lmax)
    node = Irreps(f"{mul}x0e") if layer0 else Irreps(
        "+".join(f"{mul}x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1)))
    target = (sh_ir * mul).sort()[0].simplify()
    idx, info = _lib.tp_config_by_sig(cg.fnv1a64(cg.tp_signature(node, sh_ir, target)))
    sh, _ = ops.edge_embed(bd.positions, csr, bd.shifts[keep.to(DEV)][csr.perm],
                           bd.edge_attr[keep.to(DEV)][csr.perm].reshape(-1), lmax, 6, 0.6, rmax)
    torch.manual_seed(6)
    n, e = csr.num_nodes, csr.num_edges
    x = torch.randn(n, info["din"], device=DEV)
    w = torch.randn(e, info["wn"], device=DEV)
    w = w.to(torch.bfloat16) if bf else w
    g = torch.randn(n, info["dmid"], device=DEV)
    saved = ops.TP_BWD_SENDER
    out = {}
    try:
        for flag in (True, False):
            ops.TP_BWD_SENDER = flag
            xx = x.clone().requires_grad_(True)
            ww = w.clone().requires_grad_(True)
            (ops.tp_interaction(xx, sh, ww, csr, idx, info, 0.25) * g).sum().backward()
            out[flag] = (xx.grad, ww.grad)
    finally:
        ops.TP_BWD_SENDER = saved
    (gxs, gws), (gxe, gwe) = out[True], out[False]
    assert gxs.dtype == torch.float32 and gws.dtype == w.dtype
    assert rel_err(gws, gwe) < (2 ** -8 if bf else 1e-6)
    assert float(gxs[:7].abs().max()) == 0.0
    assert rel_err(gxs, gxe) < (1e-2 if bf else 1e-6)


@pytest.mark.parametrize("bf", [False, True])
def test_torch_library_tp_interaction_matches_autograd_path(bf):
    """torch.ops.eelg.tp_interaction (+ its registered autograd) vs ops.tp_interaction: the same
    kernels in the same order -> bitwise; torch.library.opcheck on schema, fake tensor and
    autograd registration."""
    from gnn import _lib, ops, torch_ops  # noqa: F401
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    csr = ops.EdgeCSR.build(bd.edge_index, b.node_attrs.shape[0])
    idx, info, _ = _lib.tp_config("tpB_l4")
    sh, _ = ops.edge_embed(bd.positions, csr, bd.shifts[csr.perm],
                           bd.edge_attr[csr.perm].reshape(-1), 4, 6, 0.6, rmax)
    torch.manual_seed(7)
    x = torch.randn(csr.num_nodes, info["din"], device=DEV)
    w = torch.randn(csr.num_edges, info["wn"], device=DEV)
    w = w.to(torch.bfloat16) if bf else w
    g = torch.randn(csr.num_nodes, info["dmid"], device=DEV)
    cargs = (csr.sender, csr.receiver, csr.rowptr, csr.sperm, csr.srowptr)
    x1, w1 = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    a1 = torch.ops.eelg.tp_interaction(x1, sh, w1, *cargs, idx, 0.25)
    (a1 * g).sum().backward()
    x2, w2 = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    a2 = ops.tp_interaction(x2, sh, w2, csr, idx, info, 0.25)
    (a2 * g).sum().backward()
    assert torch.equal(a1, a2) and torch.equal(x1.grad, x2.grad) and torch.equal(w1.grad, w2.grad)
    torch.library.opcheck(torch.ops.eelg.tp_interaction.default,
                          (x.clone().requires_grad_(True), sh, w, *cargs, idx, 0.25),
                          test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))


@pytest.mark.parametrize("bf", [False, True])
def test_tp_bwd_sender_position_store_is_bitwise(bf):
    """eelg_tp_bwd_sorted (gxe rows stored at their sender-order position, contiguous sender
    sum) vs eelg_tp_bwd + the sperm-gathering sender sum: same values summed in the same order
    -> bitwise equal grad_x and grad_w."""
    from gnn import _lib, ops
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    csr = ops.EdgeCSR.build(bd.edge_index, b.node_attrs.shape[0])
    idx, info, _ = _lib.tp_config("tpB_l4")
    sh, _ = ops.edge_embed(bd.positions, csr, bd.shifts[csr.perm],
                           bd.edge_attr[csr.perm].reshape(-1), 4, 6, 0.6, rmax)
    torch.manual_seed(8)
    x = torch.randn(csr.num_nodes, info["din"], device=DEV)
    w = torch.randn(csr.num_edges, info["wn"], device=DEV)
    w = w.to(torch.bfloat16) if bf else w
    g = torch.randn(csr.num_nodes, info["dmid"], device=DEV)
    saved = (ops.TP_BWD_SPOS, ops.TP_BWD_SENDER)
    out = {}
    try:
        ops.TP_BWD_SENDER = False
        for flag in (True, False):
            ops.TP_BWD_SPOS = flag
            xx, ww = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
            (ops.tp_interaction(xx, sh, ww, csr, idx, info, 0.25) * g).sum().backward()
            out[flag] = (xx.grad, ww.grad)
    finally:
        ops.TP_BWD_SPOS, ops.TP_BWD_SENDER = saved
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])
