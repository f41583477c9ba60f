import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "energy-equiv-lattice-gnn_amd"); sys.path.insert(0, ".")
from helpers import batch, batch_to, copy_params, params
import oracle.model as omodel
from oracle.train import stiffness_loss as oracle_loss
from gnn.model import EnergyEquivGNN
from gnn.train import stiffness_loss
def rel_err(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
b, rmax = batch(4, 50, 200, 1234)
bd = b.to("cuda")
p = params(2, lmax=4, max_edge_radius=rmax)
torch.manual_seed(0)
o = omodel.EnergyEquivGNN(p).double()
bo = batch_to(b, "cpu", torch.float64)
co = o(bo)["stiffness"]; lo = oracle_loss(co, bo.stiffness); lo.backward()
po = dict(o.named_parameters())
for sd in ("float32", "bfloat16"):
    p.storage_dtype = sd
    m = EnergyEquivGNN(p).to("cuda"); copy_params(o, m)
    cm = m(bd)["stiffness"]; lm = stiffness_loss(cm, bd.stiffness); lm.backward()
    print(sd, "stiff", rel_err(cm, co), "loss", abs(lm.item()-lo.item())/abs(lo.item()))
    errs = sorted(((rel_err(pm.grad, po[n].grad), n, float(po[n].grad.abs().max())) for n, pm in m.named_parameters()), reverse=True)
    for e in errs[:8]: print("  ", e)
