"""Hidden irreps with 16 and 64 channels per l (the reference takes any
``hidden_irreps``, ``gnn/model.py:31-39``).  The generated interaction kernels run one half-wave
per 32 channels: mul = 64 is two channel groups on the grid, mul = 16 leaves lanes 16..31 of a
half-wave without a channel; the contraction kernels take mul / 4 channel quads per node tile.

Tolerances as tests/test_gpu_parity.py: stiffness and loss within 1e-4 of the fp64 oracle,
every parameter gradient within 1e-5 of its own largest entry; the interaction block within
1e-5 (output, grad-x, parameter gradients)."""
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


@pytest.mark.parametrize("mul,lmax,correlation", [(16, 4, 3), (64, 4, 3), (16, 2, 2), (64, 3, 1),
                                                  (64, 1, 3)])
def test_model_with_other_channel_counts_matches_oracle(mul, lmax, correlation):
    from gnn.model import EnergyEquivGNN
    from gnn.train import stiffness_loss
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    p = params(2, lmax=lmax, max_edge_radius=rmax, correlation=correlation,
               hidden_irreps=_hidden(lmax, mul))
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
    po = dict(o.named_parameters())
    worst = max(rel_err(pm.grad, po[name].grad) for name, pm in m.named_parameters())
    record_parity(f"model_mul{mul}_l{lmax}_c{correlation}", stiffness=rel_err(cm, co),
                  loss=abs(lm.item() - lo.item()) / abs(lo.item()), grad_params=worst)
    assert rel_err(cm, co) < 1e-4
    assert abs(lm.item() - lo.item()) <= 1e-4 * abs(lo.item())
    assert worst < 1e-5


@pytest.mark.parametrize("mul,layer_index", [(16, 0), (16, 1), (64, 0), (64, 1)])
def test_interaction_block_other_channel_counts(mul, layer_index):
    from gnn.model import EnergyEquivGNN
    b, rmax = batch(4, 50, 200, 1234)
    bd = b.to(DEV)
    p = params(2, hidden_irreps=_hidden(4, mul))
    torch.manual_seed(0)
    o = omodel.EnergyEquivGNN(p).double()
    m = EnergyEquivGNN(p).to(DEV)
    copy_params(o, m)
    o_int = o.stiffness_head.layers[layer_index].interaction
    m_int = m.stiffness_head.layers[layer_index].interaction
    n = b.node_attrs.shape[0]
    torch.manual_seed(1)
    x = torch.randn(n, o_int._node_feats_irreps.dim, dtype=torch.float64)
    vec, ln = omace.get_edge_vectors_and_lengths(b.positions.double(), b.edge_index, b.shifts.double())
    sh = oo3.spherical_harmonics(4, vec)
    ef = torch.cat([oo3.soft_one_hot_linspace(ln.squeeze(-1), 0, 0.6, 6),
                    oo3.soft_one_hot_linspace(b.edge_attr.double().squeeze(-1), 0, rmax, 6)], 1)
    xo = x.clone().requires_grad_(True)
    yo, _ = o_int(xo, sh, ef, b.edge_index)
    go = torch.randn_like(yo)
    (yo * go).sum().backward()
    xm = x.float().to(DEV).requires_grad_(True)
    ym, _ = m_int(xm, sh.float().to(DEV), ef.float().to(DEV), bd.edge_index)
    (ym * go.float().to(DEV)).sum().backward()
    po = dict(o_int.named_parameters())
    gerr = {name: rel_err(pm.grad, po[name].grad) for name, pm in m_int.named_parameters()}
    assert rel_err(ym, yo) < 1e-5
    assert rel_err(xm.grad, xo.grad) < 1e-5
    for name, e in gerr.items():
        assert e < 1e-5, name
