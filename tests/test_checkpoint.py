"""Reference checkpoint compatibility (CPU; SURVEY.md section 5 'Checkpoint / resume').

The reference's ``state_dict`` holds, besides the parameters, the persistent buffers
``Contraction.U_matrix_{1,2,3}`` (``gnn/mace.py:198-205``), ``Cart_4_to_Mandel.mask/rows/cols``
(``gnn/blocks.py:401-417``) and ``Spherical_to_Cartesian.Q_flat`` (``:427-436``).  The oracle
registers the same buffers, so its ``state_dict`` stands in for a reference checkpoint.
"""
import pytest
import torch

import oracle.model as omodel
from gnn import cg
from gnn.model import EnergyEquivGNN

from helpers import params


def _pair(layers=2, lmax=4):
    p = params(layers, lmax=lmax)
    torch.manual_seed(0)
    return omodel.EnergyEquivGNN(p), EnergyEquivGNN(p)


@pytest.mark.parametrize("lmax", [3, 4])
def test_state_dict_round_trips_strictly_both_ways(lmax):
    o, m = _pair(2, lmax)
    so, sm = o.state_dict(), m.state_dict()
    assert set(so) == set(sm)
    for k in so:
        assert so[k].shape == sm[k].shape, k
        if "U_matrix" in k or k.endswith(("mask", "rows", "cols")):
            assert torch.allclose(so[k].double(), sm[k].double(), atol=1e-7), k
    m.load_state_dict(so, strict=True)
    for k, v in m.named_parameters():
        assert torch.equal(v, dict(o.named_parameters())[k]), k
    o.load_state_dict(m.state_dict(), strict=True)


def _rotate_U_basis(sd, key_prefix, nu, seed):
    """U -> U R and W -> R^T W for a random orthogonal R: the same contraction in another
    basis of the (l, nu) path space, as a reference built with other conventions would hold."""
    u = sd[f"{key_prefix}.U_matrix_{nu}"]
    w = sd[f"{key_prefix}.weights.{nu}"]
    k = u.shape[-1]
    g = torch.Generator().manual_seed(seed)
    r, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    if k == 1:
        r = -torch.ones(1, 1, dtype=torch.float64)      # a sign flip, the only change for K = 1
    sd[f"{key_prefix}.U_matrix_{nu}"] = (u.double() @ r).float()
    sd[f"{key_prefix}.weights.{nu}"] = (r.T @ w.double()).float()


def test_U_in_another_basis_is_adopted():
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sc_key = "stiffness_head.layers.1.product.symmetric_contractions"
    before = m.stiffness_head.layers[1].product.symmetric_contractions
    m.load_state_dict(sd, strict=True)
    coef_ref = before.coefficients().double()
    for name, nu, seed in (("32x2e", 3, 1), ("32x4e", 2, 2), ("32x0e", 3, 3), ("32x1o", 1, 4)):
        _rotate_U_basis(sd, f"{sc_key}.contractions.{name}", nu, seed)
    m.load_state_dict(sd, strict=True)
    sc = m.stiffness_head.layers[1].product.symmetric_contractions
    assert len(sc._u_loaded) == 4
    coef = sc.coefficients().double()
    assert float(((coef - coef_ref).abs().max() / coef_ref.abs().max()).detach()) < 1e-5
    # the adopted basis is what the model now saves
    again = m.state_dict()
    key = f"{sc_key}.contractions.32x2e.U_matrix_3"
    assert torch.equal(again[key], sd[key])
    # and the oracle with the rotated checkpoint agrees with the original oracle
    o2 = omodel.EnergyEquivGNN(params(2, lmax=4))
    o2.load_state_dict(sd, strict=True)


def test_unrepresentable_U_is_refused():
    o, m = _pair(2, 4)
    sd = o.state_dict()
    key = "stiffness_head.layers.1.product.symmetric_contractions.contractions.32x2e.U_matrix_2"
    g = torch.Generator().manual_seed(5)
    sd[key] = sd[key] + 0.1 * torch.randn(sd[key].shape, generator=g)
    with pytest.raises(RuntimeError, match="do not evaluate"):
        m.load_state_dict(sd, strict=True)


def test_mandel_tables_are_verified():
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sd["stiffness_head.cart_to_Mandel.mask"] = sd["stiffness_head.cart_to_Mandel.mask"] * 2
    with pytest.raises(RuntimeError, match="Cart_4_to_Mandel"):
        m.load_state_dict(sd, strict=True)


def test_loaded_Q_flat_is_used():
    """``Q_flat`` (e3nn's ReducedTensorProducts basis in the reference) is a real buffer: a
    checkpoint's change of basis replaces the derived one."""
    o, m = _pair(2, 4)
    sd = o.state_dict()
    g = torch.Generator().manual_seed(6)
    r, _ = torch.linalg.qr(torch.randn(21, 21, generator=g, dtype=torch.float64))
    sd["stiffness_head.sph_to_cart.Q_flat"] = (r @ sd["stiffness_head.sph_to_cart.Q_flat"].double()).float()
    m.load_state_dict(sd, strict=True)
    assert torch.equal(m.stiffness_head.sph_to_cart.Q_flat, sd["stiffness_head.sph_to_cart.Q_flat"])


# e3nn 0.5's derived buffers in a reference checkpoint (gnn/blocks.py:516-535,553-559,268-279):
# output masks of every Linear / TensorProduct / the Gate's ElementwiseTensorProduct, empty
# ``weight`` placeholders of the external-weight tensor products, empty ``bias`` placeholders
# of the bias-less Linears
E3NN_KEYS = {
    "stiffness_head.layers.1.interaction.linear_up.output_mask": (800,),
    "stiffness_head.layers.1.interaction.linear_up.bias": (0,),
    "stiffness_head.layers.1.interaction.conv_tp.output_mask": (7360,),
    "stiffness_head.layers.1.interaction.conv_tp.weight": (0,),
    "stiffness_head.layers.1.interaction.linear.output_mask": (800,),
    "stiffness_head.layers.1.product.linear.output_mask": (800,),
    "stiffness_head.layers.1.product.linear.bias": (0,),
    "stiffness_head.layers.0.interaction.conv_tp.weight": (0,),
    "stiffness_head.nonlin_readout.linear_1.bias": (0,),
    "stiffness_head.nonlin_readout.linear_2.bias": (0,),
    "stiffness_head.nonlin_readout.equivariant_nonlin.mul.output_mask": (768,),
    "stiffness_head.nonlin_readout.equivariant_nonlin.mul.weight": (0,),
    "stiffness_head.linear.output_mask": (21,),
}


def test_e3nn_buffers_are_emitted_and_accepted():
    """Both the oracle (the stand-in for a reference checkpoint) and the product carry every
    e3nn derived buffer under the reference's names; a strict load accepts them."""
    o, m = _pair(2, 4)
    so, sm = o.state_dict(), m.state_dict()
    for k, shape in E3NN_KEYS.items():
        assert tuple(so[k].shape) == shape, k
        assert tuple(sm[k].shape) == shape, k
        assert torch.equal(so[k], sm[k].to(so[k].dtype)), k
    m.load_state_dict(so, strict=True)
    o.load_state_dict(sm, strict=True)


def test_e3nn_output_masks_are_verified():
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sd["stiffness_head.layers.1.interaction.linear.output_mask"] = torch.zeros(800)
    with pytest.raises(RuntimeError, match="output mask"):
        m.load_state_dict(sd, strict=True)


@pytest.mark.parametrize("key", ["stiffness_head.layers.1.interaction.conv_tp.weight",
                                 "stiffness_head.layers.1.interaction.linear_up.bias",
                                 "stiffness_head.nonlin_readout.equivariant_nonlin.mul.weight"])
def test_e3nn_placeholders_must_be_empty(key):
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sd[key] = torch.ones(3)
    with pytest.raises(RuntimeError, match="placeholder"):
        m.load_state_dict(sd, strict=True)


def test_standard_checkpoint_after_rotated_one_restores_the_derived_basis():
    """loading a checkpoint with U in another basis, then a standard one, must
    compute with the derived U again (and save it)."""
    o, m = _pair(2, 4)
    std = o.state_dict()
    sc_key = "stiffness_head.layers.1.product.symmetric_contractions"
    m.load_state_dict(std, strict=True)
    sc = m.stiffness_head.layers[1].product.symmetric_contractions
    coef_std = sc.coefficients().detach().clone()
    u_std = sc.u_sym.clone()
    rot = {k: v.clone() for k, v in std.items()}
    _rotate_U_basis(rot, f"{sc_key}.contractions.32x2e", 3, 1)
    m.load_state_dict(rot, strict=True)
    assert len(sc._u_loaded) == 1 and not torch.equal(sc.u_sym, u_std)
    m.load_state_dict(std, strict=True)
    assert sc._u_loaded == {}
    assert torch.equal(sc.u_sym, u_std)
    assert torch.equal(sc.coefficients().detach(), coef_std)
    key = f"{sc_key}.contractions.32x2e.U_matrix_3"
    assert torch.allclose(m.state_dict()[key].double(), std[key].double(), atol=1e-7)


def test_failed_U_load_leaves_the_basis_untouched():
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sc = m.stiffness_head.layers[1].product.symmetric_contractions
    u0 = sc.u_sym.clone()
    sc_key = "stiffness_head.layers.1.product.symmetric_contractions.contractions"
    _rotate_U_basis(sd, f"{sc_key}.32x2e", 3, 1)                     # adoptable
    sd[f"{sc_key}.32x4e.U_matrix_1"] = torch.zeros(3, 3)               # bad shape
    with pytest.raises(RuntimeError):
        m.load_state_dict(sd, strict=True)
    assert torch.equal(sc.u_sym, u0)


def test_checkpoint_without_mandel_tables_loads():
    """checkpoints written before Cart_4_to_Mandel registered its tables."""
    o, m = _pair(2, 4)
    sd = m.state_dict()
    for name in ("mask", "rows", "cols"):
        del sd[f"stiffness_head.cart_to_Mandel.{name}"]
    m.load_state_dict(sd, strict=True)


def test_reference_U_shapes():
    assert cg.reference_U_shape("0e+1o+2e+3o+4e", 0, 3) == (25, 25, 25, 42)
    assert cg.reference_U_shape("0e+1o+2e+3o+4e", 4, 3) == (9, 25, 25, 25, 150)
    assert cg.reference_U_shape("0e+1o+2e+3o+4e", 0, 1) == (25, 1)


def test_weights_only_partial_load_keeps_an_adopted_basis():
    """a ``strict=False`` load carrying no U buffers (weights only) must not reset
    an adopted U basis: the coefficients, hence the outputs, stay the same."""
    o, m = _pair(2, 4)
    sd = o.state_dict()
    sc_key = "stiffness_head.layers.1.product.symmetric_contractions"
    _rotate_U_basis(sd, f"{sc_key}.contractions.32x2e", 3, 1)
    m.load_state_dict(sd, strict=True)
    sc = m.stiffness_head.layers[1].product.symmetric_contractions
    u_adopted = sc.u_sym.clone()
    coef = sc.coefficients().detach().clone()
    weights_only = {k: v for k, v in sd.items() if "U_matrix" not in k}
    m.load_state_dict(weights_only, strict=False)
    assert len(sc._u_loaded) == 1
    assert torch.equal(sc.u_sym, u_adopted)
    assert torch.equal(sc.coefficients().detach(), coef)
