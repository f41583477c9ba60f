#!/usr/bin/env python3
"""torch-level glue ops of the bench training step grouped by op and input shapes (device
time), to find the elementwise / reduction launches around the HIP kernels.
Usage: python tools/torchprof_shapes.py [--steps 2]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    import bench
    from gnn import EnergyEquivGNN
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    ds = SyntheticLattices(32, 1024, 4096, 1234)
    batch = collate([ds[g] for g in range(32)]).to("cuda")
    params = bench.make_params(4, ds.max_edge_radius)
    torch.manual_seed(0)
    model = EnergyEquivGNN(params).cuda()
    model.edge_graph(batch)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, fused=True)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], batch.stiffness)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 10.0)
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
    for e in rows[:45]:
        print(f"{e.self_device_time_total / args.steps:9.1f} us/step {e.count / args.steps:5.1f}x "
              f"{e.key:28s} {str(e.input_shapes)[:110]}")


if __name__ == "__main__":
    main()
