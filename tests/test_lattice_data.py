"""Lattice data path (CPU): catalogue entry -> Data -> RotateLat -> collate + CSR
(gnn/datasets.py:112-248, scripts/train_utils.py:114-146).  The 'lattices' helpers are
absent from the reference, so these are property checks of our restatement (unpinned)."""
import math

import numpy as np
import pytest
import torch

from gnn.lattice_data import (GLAMM_Dataset, RotateLat, cart4_to_mandel, mandel_to_cart4,
                              mandel_to_voigt, process_lattice, rand_rotation, transform_matrix,
                              unit_cell_volume, voigt_to_mandel)


def iso_mandel(lam=1.3, mu=0.7):
    m = np.zeros((6, 6))
    m[:3, :3] = lam
    m[:3, :3] += 2 * mu * np.eye(3)
    m[3:, 3:] = 2 * mu * np.eye(3)
    return m


def bcc_entry(rho=(0.01, 0.02, 0.05)):
    """body-centred cubic strut lattice in reduced coordinates: corner node 0, centre node 1,
    8 struts centre -> corners (with their periodic image offsets); an unused node 2."""
    nodes = [[0, 0, 0], [0.5, 0.5, 0.5], [0.25, 0.25, 0.25]]
    adj, tess = [], []
    for sx in (0, 1):
        for sy in (0, 1):
            for sz in (0, 1):
                adj.append([1, 0])
                tess.append([sx, sy, sz])
    s = np.linalg.inv(iso_mandel())
    return {"name": "bcc", "reduced_node_coordinates": nodes, "fundamental_edge_adjacency": adj,
            "fundamental_tesselation_vecs": tess, "lattice_constants": [2.0, 2.0, 2.0, 90, 90, 90],
            "compliance_tensors_M": {r: s * (1 + r) for r in rho}}


def test_mandel_cart4_roundtrip_and_model_convention():
    from gnn.blocks import Cart_4_to_Mandel
    m = np.random.default_rng(0).normal(size=(6, 6))
    m = m + m.T
    c = mandel_to_cart4(m)
    assert np.allclose(cart4_to_mandel(c), m)
    # the model's own Cart_4_to_Mandel (reference gnn/blocks.py:392-425) agrees
    got = Cart_4_to_Mandel()(torch.tensor(c, dtype=torch.float32)[None])[0].numpy()
    assert np.allclose(got, m, atol=1e-5)
    # minor/major symmetry of the cartesian tensor
    assert np.allclose(c, c.transpose(1, 0, 2, 3)) and np.allclose(c, c.transpose(2, 3, 0, 1))


def test_voigt_mandel_conversions():
    c_m = iso_mandel()
    c_v = mandel_to_voigt(c_m, "stiffness")
    assert np.allclose(c_v[3:, 3:], 0.7 * np.eye(3))          # Voigt C44 = mu
    s_v = np.linalg.inv(c_v)
    assert np.allclose(voigt_to_mandel(s_v, "compliance"), np.linalg.inv(c_m))
    assert np.allclose(voigt_to_mandel(c_v, "stiffness"), c_m)


def test_transform_matrix_and_volume():
    q = transform_matrix([1.0, 2.0, 3.0, 90, 90, 90])
    assert np.allclose(q, np.diag([1, 2, 3]))
    q = transform_matrix([1.0, 1.0, 1.0, 60, 60, 60])             # rhombohedral: unit vectors
    assert np.allclose(np.linalg.norm(q, axis=0), 1.0)
    assert abs(abs(np.linalg.det(q)) - unit_cell_volume([1, 1, 1, 60, 60, 60])) < 1e-12
    assert abs(unit_cell_volume([1.0, 2.0, 3.0, 90, 90, 90]) - 6.0) < 1e-12


def test_process_lattice_layout_and_radius():
    ds = process_lattice(bcc_entry(), reldens_slice=slice(None))
    assert len(ds) == 3
    d = ds[1]
    assert d.positions.shape == (2, 3) and d.node_attrs.shape == (2, 1)      # unused node dropped
    e = d.edge_index.shape[1]
    assert e == 16 and torch.equal(d.edge_index[:, :8], d.edge_index.flip(0)[:, 8:])
    assert torch.allclose(d.shifts[:8], -d.shifts[8:])
    vec = d.positions[d.edge_index[1]] - d.positions[d.edge_index[0]] + d.shifts
    assert torch.allclose(vec.norm(dim=1), torch.full((16,), math.sqrt(3.0)), atol=1e-6)
    # uniform radius with rho V = pi r^2 sum(L) over both directions
    r = math.sqrt(0.02 * 8.0 / (16 * math.sqrt(3.0) * math.pi))
    assert torch.allclose(d.edge_attr, torch.full((16, 1), r), rtol=1e-6)
    assert d.stiffness.shape == (1, 3, 3, 3, 3) and d.rel_dens == 0.02
    assert np.allclose(cart4_to_mandel(d.stiffness[0].numpy()), iso_mandel() / 1.02)


def test_rotate_lat_preserves_invariants_and_geometry():
    d = process_lattice(bcc_entry())[0]
    q = rand_rotation(torch.Generator().manual_seed(3), dtype=torch.float64)
    r = RotateLat()(d, Q=q)
    assert r.stiffness.shape == (1, 6, 6)
    ev0 = torch.linalg.eigvalsh(torch.tensor(cart4_to_mandel(d.stiffness[0].numpy())))
    ev1 = torch.linalg.eigvalsh(r.stiffness[0].double())
    assert torch.allclose(ev0, ev1, atol=1e-9)
    assert torch.allclose(r.positions.double(), d.positions.double() @ q.T, atol=1e-6)
    v0 = d.positions[d.edge_index[1]] - d.positions[d.edge_index[0]] + d.shifts
    v1 = r.positions[r.edge_index[1]] - r.positions[r.edge_index[0]] + r.shifts
    assert torch.allclose(v0.norm(dim=1), v1.norm(dim=1), atol=1e-5)
    with pytest.raises(AssertionError):
        RotateLat(rotate=False)(d, Q=q)


def test_dataset_collate_with_csr_and_scaling():
    from gnn.data import collate
    ds = GLAMM_Dataset([bcc_entry(), dict(bcc_entry(), name="bcc2")], n_reldens=2, transform=RotateLat())
    assert len(ds) == 4
    ds.scale_targets(reldens_norm=True)
    b = collate([ds[i] for i in range(4)])
    assert b.stiffness.shape == (4, 6, 6) and b.num_graphs == 4
    assert torch.is_tensor(b.rel_dens) and b.rel_dens.shape == (4,)
    assert b.name == ["bcc", "bcc", "bcc2", "bcc2"]
    assert b.csr["rowptr"].shape == (9,) and int(b.csr["rowptr"][-1]) == 64
    with pytest.raises(NotImplementedError):
        GLAMM_Dataset(catalogue_path="x.lat")


def test_explicit_edge_radii_and_voigt_input():
    e = bcc_entry(rho=(0.01,))
    e.pop("compliance_tensors_M")
    c_v = mandel_to_voigt(iso_mandel(), "stiffness")
    e["compliance_tensors_V"] = {0.01: np.linalg.inv(c_v)}
    e["fundamental_edge_radii"] = {0.010000001: [0.03] * 8}
    d = process_lattice(e, edge_ft_format="r,L", graph_ft_format="Mandel")[0]
    assert torch.allclose(d.edge_attr[:, 0], torch.full((16,), 0.03))
    assert torch.allclose(d.edge_attr[:, 1], torch.full((16,), math.sqrt(3.0)), atol=1e-6)
    assert np.allclose(d.stiffness[0].numpy(), iso_mandel())
