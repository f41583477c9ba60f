#!/usr/bin/env python3
"""Host-side cost of the bench training step: wall time of each step() call as the host
enqueues it (no synchronisation), against the synchronised per-step time.  If the enqueue time
approaches the GPU time, the step is host-bound and the GPU queue runs dry between kernels.
usage (GPU box): python tools/hosttime.py [--steps 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--model", default="egnn", choices=["egnn", "cgc_modified", "cgc_vanilla"])
    args = ap.parse_args()
    import bench
    from gnn import EnergyEquivGNN
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    if args.model == "egnn":
        ds = SyntheticLattices(32, 1024, 4096, 1234)
        mine = [ds[g] for g in range(32)]
        params = bench.make_params(4, max(float(d.edge_attr.max()) for d in mine))
        torch.manual_seed(0)
        model = EnergyEquivGNN(params).cuda()
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, fused=True)
        batch = collate(mine).to("cuda")
        target = batch.stiffness
    else:   # bench.main_cgc's model, batch and optimizer (256 graphs)
        from argparse import Namespace
        from gnn import cgc
        modified = args.model == "cgc_modified"
        p = Namespace(hidden_irreps=128 if modified else 64, interaction_reduction="sum",
                      global_reduction="mean", message_passes=3, positive="square")
        ds = SyntheticLattices(256, 1024, 4096, 1234)
        batch = collate([ds[g] for g in range(256)]).to("cuda")
        torch.manual_seed(0)
        model = (cgc.CrystGraphConv if modified else cgc.CrystGraphConvVanilla)(p).cuda()
        iu = torch.triu_indices(6, 6)
        target = batch.stiffness if modified else batch.stiffness[:, iu[0], iu[1]]
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, weight_decay=1e-8)
    EnergyEquivGNN.edge_graph(batch)
    plist = list(model.parameters())

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], target)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(plist, 10.0)
        opt.step()
        return loss

    parts = {"forward": 0.0, "backward": 0.0, "clip+adamw": 0.0}

    def step_parts():
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], target)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        torch.nn.utils.clip_grad_norm_(plist, 10.0)
        opt.step()
        t3 = time.perf_counter()
        parts["forward"] += t1 - t0
        parts["backward"] += t2 - t1
        parts["clip+adamw"] += t3 - t2

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / args.steps
    # host enqueue time per step: each step after a full drain, so the host never waits on a
    # full queue; the host time is measured before the synchronisation
    host = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        step_parts()
        host.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    host.sort()
    n = args.steps
    print(f"synchronised step {gpu * 1e3:.3f} ms; host enqueue per step median {host[n // 2] * 1e3:.3f} ms "
          f"(min {host[0] * 1e3:.3f}); " + ", ".join(f"{k} {v / n * 1e3:.3f} ms" for k, v in parts.items()))


if __name__ == "__main__":
    main()
