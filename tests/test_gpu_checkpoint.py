"""A reference-format checkpoint drives the HIP model to the reference's outputs.

The fp64 oracle's ``state_dict`` (same keys and buffers as the reference's, including the
``U_matrix_*`` tensors) is loaded with ``strict=True``; the HIP forward and loss must then
match the oracle at 1e-4 -- also after the checkpoint's contraction bases have been
rotated (U -> U R, W -> R^T W), which the HIP model must adopt rather than ignore."""
import pytest
import torch

import oracle.model as omodel
from oracle.train import stiffness_loss as oracle_loss

from helpers import batch, batch_to, params
from test_checkpoint import _rotate_U_basis

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("rotate", [False, True])
def test_oracle_checkpoint_loads_strictly_and_matches(rotate):
    from gnn.model import EnergyEquivGNN
    from gnn.train import stiffness_loss
    b, rmax = batch(4, 50, 200, 99)
    p = params(2, lmax=4, max_edge_radius=rmax)
    torch.manual_seed(3)
    o = omodel.EnergyEquivGNN(p).double()
    sd = {k: v.float() if v.is_floating_point() else v for k, v in o.state_dict().items()}
    if rotate:
        for layer in (0, 1):
            pre = f"stiffness_head.layers.{layer}.product.symmetric_contractions.contractions"
            for i, name in enumerate(("32x0e", "32x1o", "32x2e", "32x3o", "32x4e")):
                for nu in (1, 2, 3):
                    _rotate_U_basis(sd, f"{pre}.{name}", nu, 100 * layer + 10 * i + nu)
        o.load_state_dict(sd, strict=True)       # the oracle runs the rotated checkpoint too
        o = o.double()
    torch.manual_seed(12345)                     # a different init: everything must come from sd
    m = EnergyEquivGNN(p)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    bo = batch_to(b, "cpu", torch.float64)
    co = o(bo)["stiffness"]
    lo = oracle_loss(co, bo.stiffness)
    bd = b.to(DEV)
    with torch.no_grad():
        cm = m(bd)["stiffness"]
        lm = stiffness_loss(cm, bd.stiffness)
    assert rel_err(cm, co) < 1e-4
    assert abs(lm.item() - lo.item()) <= 1e-4 * abs(lo.item())
