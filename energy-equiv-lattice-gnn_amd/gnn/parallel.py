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
    """One flat buffer for all gradients; ``__call__`` all-reduces and averages them.

    Packing is one ``torch.cat`` and unpacking one ``_foreach_copy_`` (a handful of
    launches instead of two copies per parameter), so the exchange costs one RCCL
    all-reduce plus O(1) kernels per step.  A parameter without a gradient on this rank
    contributes zeros (one cached zero tensor, no per-step fill) and receives a copy of the
    averaged slice."""

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.numel = sum(p.numel() for p in self.params)
        self.group = group

    def __call__(self) -> None:
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1 or not self.params:
            return
        if not hasattr(self, "_zeros"):
            self._zeros = {}
        parts = []
        for p in self.params:
            if p.grad is not None:
                parts.append(p.grad.reshape(-1))
            else:
                z = self._zeros.get(id(p))
                if z is None or z.device != p.device:
                    z = self._zeros[id(p)] = torch.zeros(p.numel(), device=p.device, dtype=p.dtype)
                parts.append(z)
        flat = torch.cat(parts)
        dist.all_reduce(flat, group=self.group)
        flat.div_(world)
        views = flat.split([p.numel() for p in self.params])
        have = [(p.grad, v.view_as(p)) for p, v in zip(self.params, views) if p.grad is not None]
        if have:
            torch._foreach_copy_([g for g, _ in have], [v for _, v in have])
        for p, v in zip(self.params, views):
            if p.grad is None:
                # a copy, not a view: a view would keep the whole flat buffer alive
                p.grad = v.view_as(p).clone()


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every replica start from rank ``src``'s weights."""
    if not dist.is_available() or not dist.is_initialized():
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)
    # writes through .data leave the version counters alone: drop the weight-derived caches
    # (the split-bf16 packed weights of o3.Linear) so the next forward re-derives them
    for m in module.modules():
        inv = getattr(m, "invalidate_packed", None)
        if inv is not None:
            inv()
