"""Golden vectors (tests/golden/config1.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces the committed outputs (pins the oracle against drift).
GPU: the HIP path reproduces them within the fp32 tolerance stated in
test_gpu_parity.py (stiffness 1e-4 relative to max|C|, loss 1e-4, grads 2e-5)."""
import os

import numpy as np
import pytest
import torch

from helpers import params

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "config1.npz")


def load():
    z = np.load(GOLDEN)          # allow_pickle=False (default): plain arrays only
    return {k: z[k] for k in z.files}


def make_batch(g, dtype):
    from gnn.data import Batch
    b = Batch()
    b.positions = torch.tensor(g["positions"], dtype=dtype)
    b.node_attrs = torch.tensor(g["node_attrs"], dtype=dtype)
    b.shifts = torch.tensor(g["shifts"], dtype=dtype)
    b.edge_attr = torch.tensor(g["edge_attr"], dtype=dtype)
    b.stiffness = torch.tensor(g["stiffness_target"], dtype=dtype)
    b.edge_index = torch.tensor(g["edge_index"])
    b.batch = torch.tensor(g["batch"])
    b.num_graphs = int(g["num_graphs"])
    return b


def set_params(model, g):
    with torch.no_grad():
        for k, p in model.named_parameters():
            p.copy_(torch.tensor(g["param/" + k]).to(p.dtype))


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double()
    a, b = a.detach(), b.detach()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def test_oracle_reproduces_golden():
    import oracle.model as omodel
    from oracle.train import stiffness_loss
    g = load()
    p = params(int(g["message_passes"]), max_edge_radius=float(g["max_edge_radius"]))
    m = omodel.EnergyEquivGNN(p).double()
    set_params(m, g)
    b = make_batch(g, torch.float64)
    c = m(b)["stiffness"]
    loss = stiffness_loss(c, b.stiffness)
    loss.backward()
    assert rel(c, g["out_stiffness"]) < 1e-10
    assert abs(loss.item() - float(g["out_loss"])) < 1e-10 * abs(float(g["out_loss"]))
    grads = dict(m.named_parameters())
    for k in [k[5:] for k in g if k.startswith("grad/")]:
        assert rel(grads[k].grad, g["grad/" + k]) < 1e-8, k


@pytest.mark.gpu
def test_hip_path_reproduces_golden():
    from gnn.model import EnergyEquivGNN
    from gnn.train import stiffness_loss
    g = load()
    p = params(int(g["message_passes"]), max_edge_radius=float(g["max_edge_radius"]))
    m = EnergyEquivGNN(p).to("cuda")
    set_params(m, g)
    b = make_batch(g, torch.float32).to("cuda")
    c = m(b)["stiffness"]
    loss = stiffness_loss(c, b.stiffness)
    loss.backward()
    assert rel(c, g["out_stiffness"]) < 1e-4
    assert abs(loss.item() - float(g["out_loss"])) < 1e-4 * abs(float(g["out_loss"]))
    grads = dict(m.named_parameters())
    # every parameter gradient within 2e-5 of its own largest entry (fp32 HIP vs the fp64
    # golden: reduction-order noise; the model parity tests measure <= 2.3e-6)
    worst = max(rel(grads[k].grad, g["grad/" + k]) for k in [k[5:] for k in g if k.startswith("grad/")])
    from helpers import record_parity
    record_parity("golden_config1", stiffness=rel(c, g["out_stiffness"]), grad_params=worst)
    for k in [k[5:] for k in g if k.startswith("grad/")]:
        assert rel(grads[k].grad, g["grad/" + k]) < 2e-5, k
