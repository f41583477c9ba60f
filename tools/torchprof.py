#!/usr/bin/env python3
"""Op-level breakdown of the bench training step (torch.profiler, device time by op and
by Python call site).  Usage: python tools/torchprof.py [--steps 3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=60))
    # host side: where the Python thread spends its time enqueueing the step
    print(ka.table(sort_by="self_cpu_time_total", row_limit=40, max_name_column_width=60))
    print(prof.key_averages(group_by_stack_n=4).table(sort_by="self_cuda_time_total", row_limit=30,
                                                      max_name_column_width=40, max_src_column_width=90))


if __name__ == "__main__":
    main()
