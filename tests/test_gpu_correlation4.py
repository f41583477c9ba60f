"""Correlation 4 on the device: the table-driven contraction kernels (``eelg_scg_*``,
``csrc/eelg_scg.hip``) against the fp64 oracle (the reference's ``Contraction`` with
``U_matrix_real``'s ``filter_ir_mid``, gnn/mace.py:180-280,435-477).

Tolerances as tests/test_gpu_parity.py: the product block's output, grad-x and weight gradients
within 1e-5 of their largest entry; the model's stiffness and loss within 1e-4, every parameter
gradient within 1e-5 of its own largest entry."""
import pytest
import torch

from helpers import batch, batch_to, copy_params, params, record_parity

import oracle.mace as omace
import oracle.model as omodel
import oracle.o3 as oo3
from oracle.train import stiffness_loss as oracle_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _hidden(lmax, mul):
    return "+".join(f"{mul}x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))


@pytest.mark.parametrize("lmax,mul,n", [(1, 32, 777), (2, 16, 1000)])
def test_correlation4_contraction_matches_oracle(lmax, mul, n):
    """SymmetricContraction(correlation=4) on the HIP table kernels vs the oracle: forward, grad-x
    and every weight gradient; node counts that leave partial 256-node blocks and 512-node
    coefficient chunks."""
    from gnn.mace import SymmetricContraction
    h = _hidden(lmax, mul)
    torch.manual_seed(0)
    o = omace.SymmetricContraction(oo3.Irreps(h), oo3.Irreps(h), 4).double()
    m = SymmetricContraction(h, h, 4).to(DEV)
    assert m._table is not None
    copy_params(o, m)
    x = torch.randn(n, oo3.Irreps(h).dim, dtype=torch.float64)
    xo = x.clone().requires_grad_(True)
    ref = o(omace.reshape_irreps(oo3.Irreps(h), xo))
    g = torch.randn_like(ref)
    ref.backward(g)
    xm = x.float().to(DEV).requires_grad_(True)
    out = m(xm)
    out.backward(g.float().to(DEV))
    torch.cuda.synchronize()
    po = dict(o.named_parameters())
    worst = max(rel_err(p.grad, po[k].grad) for k, p in m.named_parameters())
    record_parity(f"contraction_c4_l{lmax}_m{mul}", out=rel_err(out, ref), grad_x=rel_err(xm.grad, xo.grad),
                  grad_params=worst)
    assert rel_err(out, ref) < 1e-5
    assert rel_err(xm.grad, xo.grad) < 1e-5
    assert worst < 1e-5


def test_correlation4_lmax3_contraction_matches_fp64_table_model():
    """lmax 3 (8,238 terms): the kernels against the fp64 numpy model of their own table
    (tests/test_correlation4.py, which checks that model against the oracle's dense contraction
    at lmax 1 and the 4-slot polynomial at lmax 1-2; the oracle's own lmax-3 U build takes
    minutes).  Forward, grad-x and the weight gradients through coef = U_sym W."""
    import numpy as np
    from test_correlation4 import _table_model
    from gnn.mace import SymmetricContraction
    h = _hidden(3, 32)
    torch.manual_seed(0)
    m = SymmetricContraction(h, h, 4).to(DEV)
    tab = m._table
    n = 300
    x = torch.randn(n, m.irreps_in.dim, dtype=torch.float64)
    g = torch.randn(n, m.irreps_out.dim, dtype=torch.float64)
    coef = m.coefficients().detach().double().cpu().numpy()
    out_ref, gx_ref, gcoef = _table_model(tab, x.numpy(), coef, g.numpy())
    xm = x.float().to(DEV).requires_grad_(True)
    out = m(xm)
    out.backward(g.float().to(DEV))
    torch.cuda.synchronize()
    gw_ref = m.u_sym.double().cpu().numpy().T @ gcoef[:, :tab.desc.nterms].T      # [K, mul]
    gw = torch.cat([m.contractions[f"32x{oo3.Irrep(l, (-1) ** l)}"].weights[str(nu)].grad
                    for l, nu in m.block_order])
    e_out = rel_err(out, torch.tensor(out_ref))
    e_gx = rel_err(xm.grad, torch.tensor(gx_ref))
    e_gw = rel_err(gw, torch.tensor(gw_ref))
    record_parity("contraction_c4_l3_m32", out=e_out, grad_x=e_gx, grad_params=e_gw)
    assert e_out < 1e-5 and e_gx < 1e-5 and e_gw < 1e-5
    assert np.isfinite(gcoef).all()


@pytest.mark.parametrize("lmax", [1, 2])
def test_model_correlation4_matches_oracle(lmax):
    from gnn.model import EnergyEquivGNN
    from gnn.train import stiffness_loss
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    p = params(2, lmax=lmax, max_edge_radius=rmax, correlation=4)
    torch.manual_seed(0)
    o = omodel.EnergyEquivGNN(p).double()
    m = EnergyEquivGNN(p).to(DEV)
    copy_params(o, m)
    bo = batch_to(b, "cpu", torch.float64)
    co = o(bo)["stiffness"]
    lo = oracle_loss(co, bo.stiffness)
    lo.backward()
    cm = m(bd)["stiffness"]
    lm = stiffness_loss(cm, bd.stiffness)
    lm.backward()
    torch.cuda.synchronize()
    po = dict(o.named_parameters())
    worst = max(rel_err(pm.grad, po[name].grad) for name, pm in m.named_parameters())
    record_parity(f"model_c4_l{lmax}", stiffness=rel_err(cm, co),
                  loss=abs(lm.item() - lo.item()) / abs(lo.item()), grad_params=worst)
    assert rel_err(cm, co) < 1e-4
    assert abs(lm.item() - lo.item()) <= 1e-4 * abs(lo.item())
    assert worst < 1e-5
