"""Probe: can two ranks share one GPU over RCCL (backend 'nccl')?  Run under torch.distributed.run
with --nproc-per-node 2 on a one-GPU box; prints the all-reduce result or the RCCL error."""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    t = torch.full((1024,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok, value {t[0].item()} (expect 3.0)", flush=True)
    dist.destroy_process_group()
except Exception as e:  # report, do not retry
    print(f"rank {rank}: RCCL failed: {type(e).__name__}: {str(e)[:300]}", flush=True)
    sys.exit(3)
