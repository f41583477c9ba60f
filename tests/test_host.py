"""Host-side logic (CPU): product constants vs the oracle, data path / CSR, the
generator's structural plans, and the C-ABI library (loads, exports, config
tables) -- no kernel launches."""
import math

import numpy as np
import pytest
import torch

import oracle.mace as omace
import oracle.o3 as oo3
from gnn import cg
from gnn.data import Batch, build_edge_csr, collate
from gnn.irreps import Irreps
from gnn.synthetic import SyntheticLattices, make_lattice


def test_product_cg_matches_oracle():
    for l1 in range(5):
        for l2 in range(5):
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                a = cg.wigner_3j(l1, l2, l3)
                b = oo3.wigner_3j(l1, l2, l3).numpy()
                assert np.abs(a - b).max() < 1e-12, (l1, l2, l3)


def test_product_sh_matches_oracle():
    v = np.random.default_rng(0).normal(size=(50, 3))
    a = cg.spherical_harmonics_np(4, v)
    b = oo3.spherical_harmonics(4, torch.tensor(v)).numpy()
    assert np.abs(a - b).max() < 1e-12


def test_product_u_matrices_match_oracle():
    for l in range(5):
        ir = oo3.Irreps(str(oo3.Irrep(l, (-1) ** l)))
        for nu in (1, 2, 3):
            a = cg.U_matrix("0e+1o+2e+3o+4e", l, nu)
            b = omace.U_matrix_real(oo3.Irreps("0e+1o+2e+3o+4e"), ir, nu)[-1].numpy()
            assert np.abs(a.reshape(b.shape) - b).max() < 1e-12


def test_product_change_of_basis_matches_oracle():
    assert np.abs(cg.stiffness_change_of_basis() - oo3.stiffness_change_of_basis().numpy()).max() < 1e-12


@pytest.mark.parametrize("lmax", [2, 3, 4])
def test_symcon_polynomial_equals_dense_contraction(lmax):
    """The sparse symmetrised polynomial behind the HIP kernels equals the reference's
    dense U.W contraction (gnn/mace.py:242-277)."""
    coupling = "+".join(f"{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    hid = "+".join(f"8x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    plan = cg.symcon_plan(coupling, tuple(range(lmax + 1)), 3)
    torch.manual_seed(0)
    sc = omace.SymmetricContraction(oo3.Irreps(hid), oo3.Irreps(hid), 3).double()
    ws = []
    for l, nu, k in plan.weight_blocks:
        w = sc.contractions[f"8x{oo3.Irrep(l, (-1) ** l)}"].weights[str(nu)]
        assert w.shape == (k, 8)
        ws.append(w.detach())
    coef = plan.ubig @ torch.cat(ws).numpy()
    D = plan.D
    x = np.random.default_rng(1).normal(size=(4, 8, D))
    out = np.zeros((4, 8, D))
    for t, (nu, (a, b, c), o) in enumerate(plan.terms):
        m = x[:, :, a] * (x[:, :, b] if nu >= 2 else 1) * (x[:, :, c] if nu >= 3 else 1)
        out[:, :, o] += coef[t] * m
    with torch.no_grad():
        ref = sc(torch.tensor(x)).numpy()
    mine = np.concatenate([out[:, :, l * l:(l + 1) ** 2].reshape(4, -1) for l in range(lmax + 1)], 1)
    assert np.abs(mine - ref).max() < 1e-6 * np.abs(ref).max()


def test_irreps_sort_simplify_semantics():
    ir = Irreps("1x2e+3x0e+2x1o+1x0e")
    s, p = ir.sort()
    assert str(s) == "3x0e+1x0e+2x1o+1x2e" and p == [3, 0, 2, 1]
    assert str(s.simplify()) == "4x0e+2x1o+1x2e"
    assert (Irreps.spherical_harmonics(4) * 32).sort()[0].simplify().dim == 800


def test_synthetic_lattice_layout():
    d = make_lattice(64, 256, 5)
    ei = d.edge_index
    e = ei.shape[1]
    assert e == 256 and d.node_attrs.shape == (64, 1) and torch.all(d.node_attrs == 1)
    h = e // 2
    assert torch.equal(ei[:, :h], ei.flip(0)[:, h:])                 # reversed copies
    assert torch.allclose(d.shifts[:h], -d.shifts[h:])
    assert torch.equal(d.edge_attr[:h], d.edge_attr[h:])
    vec = d.positions[ei[1]] - d.positions[ei[0]] + d.shifts
    a = 0.54 * 64 ** (1 / 3)
    assert float(vec.norm(dim=-1).max()) <= math.sqrt(3) * a / 2 + 1e-5  # minimum image
    ev = torch.linalg.eigvalsh(d.stiffness[0].double())
    assert (ev > 0).all()


def test_collate_and_csr():
    ds = SyntheticLattices(3, 20, 80, 3)
    b = collate([ds[i] for i in range(3)])
    assert b.num_graphs == 3 and b.stiffness.shape == (3, 6, 6)
    assert torch.equal(b.batch, torch.repeat_interleave(torch.arange(3), 20))
    assert int(b.edge_index[:, 80:160].min()) >= 20 and int(b.edge_index[:, 80:160].max()) < 40
    assert torch.equal(b["stiffness"], b.stiffness)
    csr = build_edge_csr(b.edge_index, 60)
    recv = b.edge_index[1][csr["perm"]]
    assert torch.all(recv[1:] >= recv[:-1])
    cnt = torch.bincount(b.edge_index[1], minlength=60)
    assert torch.equal(csr["rowptr"][1:].long() - csr["rowptr"][:-1].long(), cnt)
    s = csr["sender"].long()[csr["sperm"].long()]
    assert torch.all(s[1:] >= s[:-1])
    assert torch.equal(torch.sort(csr["sperm"].long())[0], torch.arange(240))


def test_csr_handles_isolated_nodes_and_empty_graph():
    ei = torch.tensor([[0, 2], [2, 0]])
    csr = build_edge_csr(ei, 4)
    assert csr["rowptr"].tolist() == [0, 1, 1, 2, 2]
    csr0 = build_edge_csr(torch.zeros(2, 0, dtype=torch.long), 3)
    assert csr0["rowptr"].tolist() == [0, 0, 0, 0] and csr0["perm"].numel() == 0


def test_library_loads_and_exports_every_header_symbol():
    import os
    import re
    from gnn import _lib
    lib = _lib.load()
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "eelg.h")).read()
    declared = set(re.findall(r"\b(eelg_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.eelg_version().startswith(b"eelg")


def test_library_config_tables_match_host_structure():
    """Every kernel set gnn/kernel_sets.py lists is in the library under its name, with the
    structure hash the host derives (lmax 1..4, correlation 1..3, mul 16 / 32 / 64: mul 32 under
    the plain names, the others with an _m<mul> suffix)."""
    from gnn import _lib, kernel_sets
    for mul in kernel_sets.MULS:
        sfx = "" if mul == 32 else f"_m{mul}"
        for lmax in kernel_sets.LMAX:
            sh = Irreps.spherical_harmonics(lmax)
            target = (sh * mul).sort()[0].simplify()
            hid = Irreps(kernel_sets.hidden_irreps_str(lmax, mul))
            for name, node in ((f"tpA_l{lmax}{sfx}", Irreps(f"{mul}x0e")), (f"tpB_l{lmax}{sfx}", hid)):
                _, info, sig = _lib.tp_config(name)
                paths = cg.tp_paths(node, sh, target)
                assert info["din"] == node.dim and info["npaths"] == len(paths)
                assert info["wn"] == mul * len(paths) and info["nsh"] == sh.dim
                assert sig == cg.fnv1a64(cg.tp_signature(node, sh, target))
                assert _lib.tp_config_by_sig(sig)[0] == _lib.tp_config(name)[0]
    for lmax in kernel_sets.LMAX:
        coupling = kernel_sets.coupling_str(lmax)
        for corr in kernel_sets.CORRELATIONS:
            _, info, sig = _lib.sc_config(f"sc_l{lmax}_c{corr}")
            plan = cg.symcon_plan(coupling, tuple(range(lmax + 1)), corr)
            assert info["nterms"] == len(plan.terms) and info["x_row"] == 32 * plan.D
            assert info["D"] == plan.D
            assert sig == cg.fnv1a64(cg.sc_signature(coupling, tuple(range(lmax + 1)), corr))
    with pytest.raises(_lib.EELGError):
        _lib.tp_config("no_such_config")


def test_unsupported_params_fail_at_construction_with_the_supported_list():
    """params whose irreps structure has no generated kernels raise when the model is built
    (not at the first forward), naming the generated sets (gnn/kernel_sets.py)."""
    from argparse import Namespace
    from helpers import params
    from gnn.model import EnergyEquivGNN
    for change in (dict(lmax=5, hidden_irreps="32x0e+32x1o+32x2e+32x3o+32x4e+32x5o"),
                   dict(hidden_irreps="48x0e+48x1o+48x2e+48x3o+48x4e"),
                   dict(hidden_irreps="32x0e+16x1o+32x2e+32x3o+32x4e"),
                   dict(hidden_irreps="32x0e+32x1o+32x2e"),
                   dict(correlation=4)):
        p = Namespace(**{**vars(params(2)), **change})
        with pytest.raises(NotImplementedError, match="generated kernel sets"):
            EnergyEquivGNN(p)
    from gnn import kernel_sets
    for lmax in (1, 2, 3, 4):
        for corr in (1, 2, 3):
            for mul in kernel_sets.MULS:
                p = Namespace(**{**vars(params(2)), "lmax": lmax, "correlation": corr,
                                 "hidden_irreps": kernel_sets.hidden_irreps_str(lmax, mul),
                                 "readout_irreps": kernel_sets.hidden_irreps_str(lmax, 16)})
                EnergyEquivGNN(p)
    # bf16 storage of the edge tensors is generated for 32 channels only
    p = Namespace(**{**vars(params(2)), "hidden_irreps": kernel_sets.hidden_irreps_str(4, 64),
                     "storage_dtype": "bfloat16"})
    with pytest.raises(NotImplementedError, match="storage"):
        EnergyEquivGNN(p)


def test_product_rejects_cpu_tensors_loudly():
    from gnn import ops
    from gnn.o3 import Linear
    lin = Linear("4x0e", "4x0e")
    with pytest.raises(RuntimeError, match="HIP device"):
        lin(torch.randn(3, 4))


def test_product_model_param_names_match_oracle():
    from helpers import params
    from gnn.model import EnergyEquivGNN
    import oracle.model as omodel
    p = params(2)
    m, o = EnergyEquivGNN(p), omodel.EnergyEquivGNN(p)
    pm = {k: v.shape for k, v in m.named_parameters()}
    po = {k: v.shape for k, v in o.named_parameters()}
    assert pm == po
    assert sum(v.numel() for v in m.parameters()) == 223186


def test_radial_mlp_is_device_only_and_checks_shapes():
    """The radial MLP runs on the device only: the fused HIP kernels for their shapes
    (tests/test_gpu_radial.py holds their parity tests), the reference's Sequential on the
    device for other inter_MLP_dim / inter_MLP_layers; a CPU input raises either way."""
    from gnn import ops
    from gnn.blocks import TensorProductInteractionBlock
    mlp = torch.nn.Sequential(torch.nn.Linear(12, 64), torch.nn.SiLU(),
                              torch.nn.Linear(64, 40, bias=False))
    with pytest.raises(RuntimeError, match="HIP device"):
        ops.radial_mlp(torch.randn(5, 12), mlp)
    hid = "32x0e+32x1o+32x2e+32x3o+32x4e"
    sh = "1x0e+1x1o+1x2e+1x3o+1x4e"
    # shapes outside the fused kernels' set run the reference's Sequential on the device; a CPU
    # tensor still raises
    for dim, layers in ((48, 3), (64, 5), (128, 3), (16, 2)):
        blk = TensorProductInteractionBlock(hid, sh, "12x0e", hid, 4.0, MLP_dim=dim, MLP_layers=layers)
        assert not blk._radial_hip
        with pytest.raises(RuntimeError, match="HIP device"):
            blk.radial_weights(torch.randn(5, 12))
    assert TensorProductInteractionBlock(hid, sh, "12x0e", hid, 4.0, MLP_dim=32, MLP_layers=4)._radial_hip
    with pytest.raises(ValueError, match="at least one hidden layer"):
        TensorProductInteractionBlock(hid, sh, "12x0e", hid, 4.0, MLP_dim=32, MLP_layers=1)


def test_wgrad_split_k_matches_matmul():
    from gnn.ops import _wgrad
    g = torch.randn(1300, 8, dtype=torch.float64)
    x = torch.randn(1300, 5, dtype=torch.float64)
    assert torch.allclose(_wgrad(g, x, chunk=256), g.t() @ x, atol=1e-10)


def test_lmax3_with_l4_hidden_irreps_raises_like_the_reference():
    """The reference cannot build a product block whose outputs exceed the SH lmax
    (gnn/mace.py:466-476); the product says so instead of failing inside numpy."""
    from gnn.mace import SymmetricContraction
    with pytest.raises(NotImplementedError):
        SymmetricContraction("32x0e+32x1o+32x2e+32x3o", "32x0e+32x1o+32x2e+32x3o+32x4e", 3)


def test_storage_dtype_param_validation():
    """optional params.storage_dtype (BASELINE config 5): float32 default, bfloat16, else raise"""
    from gnn.model import storage_dtype
    from helpers import params
    assert storage_dtype(params(2)) == torch.float32
    assert storage_dtype(params(2, storage_dtype="bfloat16")) == torch.bfloat16
    with pytest.raises(ValueError):
        storage_dtype(params(2, storage_dtype="fp8"))


def test_torch_library_ops_fake_shapes():
    """torch.ops.eelg.* (dispatcher-visible form of the fused interaction) propagate
    shapes and dtypes on meta tensors without running HIP code."""
    from gnn import _lib, torch_ops  # noqa: F401  (registers torch.ops.eelg)
    idx, info, _ = _lib.tp_config("tpB_l4")
    n, e = 10, 40

    def meta(*s, dt=torch.float32):
        return torch.empty(*s, device="meta", dtype=dt)
    csr = [meta(e, dt=torch.int32), meta(e, dt=torch.int32), meta(n + 1, dt=torch.int32),
           meta(e, dt=torch.int32), meta(n + 1, dt=torch.int32)]
    out = torch.ops.eelg.tp_interaction(meta(n, info["din"]), meta(e, info["nsh"]),
                                        meta(e, info["wn"]), *csr, idx, 0.25)
    assert out.shape == (n, info["dmid"]) and out.dtype == torch.float32
    gx, gw = torch.ops.eelg.tp_interaction_bwd(meta(n, info["dmid"]), meta(n, info["din"]),
                                               meta(e, info["nsh"]),
                                               meta(e, info["wn"], dt=torch.bfloat16), *csr, idx, 0.25)
    assert gx.shape == (n, info["din"]) and gx.dtype == torch.float32
    assert gw.shape == (e, info["wn"]) and gw.dtype == torch.bfloat16
    assert torch.ops.eelg.segment_sum_csr(meta(e, 7), meta(n + 1, dt=torch.int32)).shape == (n, 7)


def test_readout_gate_other_than_silu_raises():
    """``GeneralNonLinearReadoutBlock(gate=...)`` (gnn/blocks.py:256,270-272): the fused Gate is
    SiLU; another activation raises instead of being replaced silently."""
    from gnn.blocks import GeneralNonLinearReadoutBlock
    hid = "32x0e+32x1o+32x2e"
    for g in (None, torch.nn.functional.silu, torch.nn.SiLU()):
        GeneralNonLinearReadoutBlock(hid, hid, "16x0e+16x1o+16x2e", gate=g)
    with pytest.raises(NotImplementedError, match="SiLU"):
        GeneralNonLinearReadoutBlock(hid, hid, "16x0e+16x1o+16x2e", gate=torch.tanh)


def test_interaction_reductions_are_accepted_and_pna_is_not():
    from gnn.blocks import TensorProductInteractionBlock
    from gnn.irreps import Irreps
    sh = Irreps.spherical_harmonics(2)
    hid = "32x0e+32x1o+32x2e"
    tgt = (sh * 32).sort()[0].simplify()
    for r in ("sum", "add", "mean", "max", "min", "mul", "MAX"):
        TensorProductInteractionBlock(hid, sh, "12x0e", tgt, 4.0, r)
    with pytest.raises(NotImplementedError, match="pna"):
        TensorProductInteractionBlock(hid, sh, "12x0e", tgt, 4.0, "pna")


def test_reshape_irreps_round_trip_matches_reference_layout():
    """``reshape_irreps`` (gnn/mace.py:316-332) and its inverse, which the product's
    ``SymmetricContraction.forward`` applies to the reference's [N, mul, 25] input."""
    from gnn.irreps import Irreps
    from gnn.mace import reshape_irreps, unreshape_irreps
    from oracle.mace import reshape_irreps as oreshape
    ir = Irreps("32x0e+32x1o+32x2e+32x3o+32x4e")
    x = torch.randn(7, ir.dim, dtype=torch.float64)
    r = reshape_irreps(ir)(x)
    assert r.shape == (7, 32, 25)
    assert torch.equal(r, oreshape("32x0e+32x1o+32x2e+32x3o+32x4e", x))
    assert torch.equal(unreshape_irreps(ir, r), x)


def test_packed_linear_rule_keeps_short_k_on_fp32_kernels():
    """The split-bf16 linear kernel is chosen only where every output slot sums K >= 128 (the
    7360 -> 800 forward); K = 32 descriptors (800 -> 800, every grad-x) stay on the fp32 kernels,
    which measured faster there (o3.LIN_X6_MINK)."""
    from gnn import o3
    big = o3.Linear("160x0e+256x1o+320x2e+320x3o+288x4e", "32x0e+32x1o+32x2e+32x3o+32x4e")
    assert big._pk_ok == {"fwd": True, "bx": False}
    sq = o3.Linear("32x0e+32x1o+32x2e+32x3o+32x4e", "32x0e+32x1o+32x2e+32x3o+32x4e")
    assert sq._pk_ok == {"fwd": False, "bx": False}


def test_morton_reorder_keeps_every_edge_vector():
    """``reorder_nodes(d, morton_order(d.positions))`` is a relabelling: node tensors are
    permuted, each edge keeps its endpoints' positions (so its vector and strut) and its order,
    and neighbours get nearby ids."""
    from gnn.data import morton_order, reorder_nodes
    d = make_lattice(600, 2400, 5)
    perm = morton_order(d.positions)
    assert torch.equal(torch.sort(perm).values, torch.arange(600))
    e = reorder_nodes(d, perm)
    assert torch.equal(e.positions, d.positions[perm]) and torch.equal(e.node_attrs, d.node_attrs[perm])
    v0 = d.positions[d.edge_index[1]] - d.positions[d.edge_index[0]]
    v1 = e.positions[e.edge_index[1]] - e.positions[e.edge_index[0]]
    assert torch.equal(v0, v1) and torch.equal(e.shifts, d.shifts) and torch.equal(e.edge_attr, d.edge_attr)
    gap = lambda g: (g.edge_index[0] - g.edge_index[1]).abs().double().mean()  # noqa: E731
    assert gap(e) < 0.5 * gap(d)


def test_bench_traffic_lookup_finds_every_workloads_roofline_kernel():
    """bench.py's roofline ``traffic`` comes from the committed PMC table under the command's
    workload key; the kernel names it looks up must match the traced names (the bf16-storage
    forward carries ``_bw``, the CGC forward is a template)."""
    import importlib.util
    import os
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("_bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    A = types.SimpleNamespace
    cases = [(A(model="egnn", batch=32, nodes=1024, edges=4096, layers=4, lmax=4, storage="float32"),
              "tp_fwd_tpB_l4"),
             (A(model="egnn", batch=32, nodes=5000, edges=20000, layers=4, lmax=3, storage="bfloat16"),
              "tp_fwd_tpB_l3_bw"),
             (A(model="cgc_modified", batch=256, nodes=1024, edges=4096), "cgc_fwd_kernel")]
    for args, kernel in cases:
        t = bench.pmc_traffic(kernel, args)
        assert t is not None and t["bytes"] > 1e9, (bench.workload_key(args), kernel)
