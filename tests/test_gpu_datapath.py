"""The data path feeding the HIP model (reference gnn/datasets.py:115-307,
scripts/train_utils.py:114-146,204-239): catalogue entries -> ``GLAMM_Dataset`` (one ``Data``
per relative density) with the ``RotateLat`` transform -> ``gnn.collate`` (receiver CSR built
at collate time) -> HIP ``EnergyEquivGNN``, against the fp64 oracle on the same ``Data``.

Tolerances as the model parity tests: stiffness and loss 1e-4 of the largest entry, every
parameter gradient 1e-5 of its own largest entry.  Equivariance through the data path: a
fixed rotation Q applied by ``RotateLat`` rotates the predicted Mandel stiffness by Q (5e-4,
the fp32 rotation tolerance of the model tests).
"""
import math

import numpy as np
import pytest
import torch

from helpers import batch_to, copy_params, params

import oracle.model as omodel
from oracle.train import stiffness_loss as oracle_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def random_entry(name, n_nodes, seed, rho=(0.01, 0.03)):
    """A periodic strut lattice in catalogue-entry form: nodes at random reduced coordinates,
    every node linked to its two nearest periodic neighbours (deduplicated), tessellation
    vectors = the integer image offsets; an SPD compliance per relative density."""
    rng = np.random.default_rng(seed)
    red = rng.random((n_nodes, 3))
    edges = {}
    for i in range(n_nodes):
        cand = []
        for j in range(n_nodes):
            for off in np.ndindex(3, 3, 3):
                o = np.asarray(off) - 1
                if j == i and not o.any():
                    continue
                cand.append((float(np.linalg.norm(red[j] + o - red[i])), j, tuple(o)))
        cand.sort()
        for _, j, o in cand[:2]:
            key = (min(i, j), max(i, j), o if i < j else tuple(-np.asarray(o)))
            edges.setdefault(key, (i, j, o))
    adj = [[i, j] for i, j, _ in edges.values()]
    tess = [list(o) for _, _, o in edges.values()]
    comp = {}
    for r in rho:
        a = rng.normal(size=(6, 6))
        comp[r] = np.linalg.inv(a @ a.T / 6 + 0.5 * np.eye(6))
    return {"name": name, "reduced_node_coordinates": red.tolist(), "fundamental_edge_adjacency": adj,
            "fundamental_tesselation_vecs": tess, "lattice_constants": [1.0, 1.2, 0.9, 90, 80, 95],
            "compliance_tensors_M": comp}


def _dataset(transform):
    from gnn.lattice_data import GLAMM_Dataset
    ents = [random_entry("a", 24, 1), random_entry("b", 31, 2), random_entry("c", 17, 3)]
    ds = GLAMM_Dataset(ents, n_reldens=2, transform=transform)
    ds.scale_targets(reldens_norm=True)
    return ds


def _pair(rmax):
    from gnn.model import EnergyEquivGNN
    p = params(2, max_edge_radius=rmax)
    torch.manual_seed(0)
    o = omodel.EnergyEquivGNN(p).double()
    m = EnergyEquivGNN(p).to(DEV)
    copy_params(o, m)
    return o, m


def test_glamm_rotatelat_collate_feeds_the_hip_model():
    from gnn.data import collate
    from gnn.lattice_data import RotateLat
    from gnn.train import stiffness_loss
    ds = _dataset(RotateLat(generator=torch.Generator().manual_seed(11)))
    data = [ds[i] for i in range(len(ds))]
    b = collate(data)
    assert b.num_graphs == 6 and b.stiffness.shape == (6, 6, 6) and "rowptr" in b.csr
    rmax = float(max(float(d.edge_attr.max()) for d in data))
    o, m = _pair(rmax)
    bo = batch_to(b, "cpu", torch.float64)
    co = o(bo)["stiffness"]
    lo = oracle_loss(co, bo.stiffness)
    lo.backward()
    bd = b.to(DEV)
    cm = m(bd)["stiffness"]
    lm = stiffness_loss(cm, bd.stiffness)
    lm.backward()
    po = dict(o.named_parameters())
    worst = max(rel_err(pm.grad, po[name].grad) for name, pm in m.named_parameters())
    assert rel_err(cm, co) < 1e-4
    assert abs(lm.item() - lo.item()) <= 1e-4 * abs(lo.item())
    assert worst < 1e-5


def test_rotatelat_rotates_the_prediction():
    """model(RotateLat(Q) d) == Q . model(d) for the predicted stiffness (in cartesian form)."""
    from gnn.data import collate
    from gnn.lattice_data import RotateLat, cart4_to_mandel, mandel_to_cart4, rand_rotation
    ds = _dataset(None)
    q = rand_rotation(torch.Generator().manual_seed(5), dtype=torch.float64)
    ident = torch.eye(3, dtype=torch.float64)
    plain = collate([RotateLat()(ds[i], Q=ident) for i in range(len(ds))])
    rot = collate([RotateLat()(ds[i], Q=q) for i in range(len(ds))])
    rmax = float(max(float(ds[i].edge_attr.max()) for i in range(len(ds))))
    _, m = _pair(rmax)
    with torch.no_grad():
        c0 = m(plain.to(DEV))["stiffness"].double().cpu().numpy()
        c1 = m(rot.to(DEV))["stiffness"].double().cpu().numpy()
    qn = q.numpy()
    want = np.stack([cart4_to_mandel(np.einsum("ijkl,ai,bj,ck,dl->abcd", mandel_to_cart4(c), qn, qn, qn, qn))
                     for c in c0])
    err = float(np.abs(c1 - want).max() / np.abs(want).max())
    assert err < 5e-4, err
