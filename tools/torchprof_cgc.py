#!/usr/bin/env python3
"""torch-level ops of the CGC benchmark step (bench.py --model cgc_modified|cgc_vanilla), grouped
by op and input shapes (device time per step), to find the glue launches around the HIP kernels.
usage (GPU box): python tools/torchprof_cgc.py [--model cgc_modified] [--steps 2]"""
import argparse
import os
import sys
from argparse import Namespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="cgc_modified", choices=["cgc_modified", "cgc_vanilla"])
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    from gnn import EnergyEquivGNN, cgc
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    modified = args.model == "cgc_modified"
    p = Namespace(hidden_irreps=128 if modified else 64, interaction_reduction="sum",
                  global_reduction="mean", message_passes=3, positive="square")
    ds = SyntheticLattices(256, 1024, 4096, 1234)
    batch = collate([ds[g] for g in range(256)]).to("cuda")
    torch.manual_seed(0)
    model = (cgc.CrystGraphConv if modified else cgc.CrystGraphConvVanilla)(p).cuda()
    iu = torch.triu_indices(6, 6)
    target = batch.stiffness if modified else batch.stiffness[:, iu[0], iu[1]]
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, weight_decay=1e-8, fused=True)
    EnergyEquivGNN.edge_graph(batch)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], target)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(model.parameters()), 10.0)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:30]:
        print(f"{e.self_device_time_total / args.steps:9.1f} us/step {e.count / args.steps:5.1f}x "
              f"{e.key:28s} {str(e.input_shapes)[:110]}")


if __name__ == "__main__":
    main()
