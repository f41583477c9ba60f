"""Graph-sharded data parallelism (one process per GPU, RCCL over xGMI).

The reference trains with Lightning's implicit DDP (``scripts/train_main.py:89-100``):
replicas, bucketed gradient all-reduce.  Here the hot path shards whole lattice
graphs across ranks (graphs are independent until the per-graph pool and loss,
SURVEY.md 8e) and exchanges exactly one thing per step: the flat fp32 gradient
(552,210 floats = 2.2 MB for the 4-layer model), all-reduced once and divided by
the world size.  On 8 GPUs that ring all-reduce moves ~3.9 MB per GPU per step,
latency-bound (~0.1 ms) against a step of tens of ms, so no bucketing/overlap is
needed.  Works with backend 'nccl' (= RCCL on ROCm) and 'gloo' (CPU tests).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import torch
import torch.distributed as dist


def shard_indices(num_items: int, rank: int, world: int, per_rank: int, step: int = 0) -> List[int]:
    """Deterministic rank-strided graph ids for one step: rank r takes the r-th
    contiguous block of ``per_rank`` graphs of the step's global batch."""
    base = step * per_rank * world + rank * per_rank
    return [(base + i) % num_items for i in range(per_rank)]


class FlatGradAllReduce:
    """One flat buffer for all gradients; ``__call__`` all-reduces and averages them."""

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.group = group

    def __call__(self) -> None:
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        off = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[off: off + n].zero_()
            else:
                self.flat[off: off + n].copy_(p.grad.reshape(-1))
            off += n
        dist.all_reduce(self.flat, group=self.group)
        self.flat.div_(world)
        off = 0
        for p in self.params:
            n = p.numel()
            g = self.flat[off: off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += n


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every replica start from rank ``src``'s weights."""
    if not dist.is_available() or not dist.is_initialized():
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)
