#!/usr/bin/env python3
"""Report host<->device synchronisations inside the bench training step
(torch.cuda.set_sync_debug_mode('warn') around steps after warm-up)."""
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402


def main():
    import bench
    from gnn import EnergyEquivGNN
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    ds = SyntheticLattices(4, 1024, 4096, 1234)
    batch = collate([ds[g] for g in range(4)]).to("cuda")
    torch.manual_seed(0)
    model = EnergyEquivGNN(bench.make_params(4, ds.max_edge_radius)).cuda()
    model.edge_graph(batch)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, fused=True)
    plist = list(model.parameters())

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], batch.stiffness)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(plist, 10.0)
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode("warn")
        step()
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print(f"{len(ws)} synchronising calls in one step")
    for w in ws[:20]:
        print(" -", str(w.message)[:160], f"({w.filename}:{w.lineno})")


if __name__ == "__main__":
    main()
