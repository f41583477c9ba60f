"""Minimal PyG-compatible ``Data`` / ``Batch`` / collate, plus the receiver- and
sender-CSR that the HIP interaction kernels traverse.

Field layout is the reference's (``gnn/datasets.py:256-269``,
``scripts/train_utils.py:135-145``): ``positions [N,3]``, ``node_attrs [N,1]``,
``edge_index [2,E]`` (row 0 = sender, row 1 = receiver, ``gnn/mace.py:345``),
``shifts [E,3]``, ``edge_attr [E,1]`` (strut radius), ``stiffness [1,6,6]``.
Collation follows PyG ~2.1 semantics: ``edge_index`` is offset by the running
node count, node/edge tensors are concatenated, ``stiffness`` is stacked to
``[B,6,6]``, and ``batch`` holds the (sorted) graph id of every node.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

_NODE_KEYS = ("positions", "node_attrs")
_EDGE_KEYS = ("shifts", "edge_attr", "unit_shifts")
_GRAPH_KEYS = ("stiffness", "compliance", "rel_dens")


class Data:
    """Attribute bag with item access (``data['stiffness']``)."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self) -> List[str]:
        return [k for k in self.__dict__ if not k.startswith("_")]

    def __getitem__(self, key):
        return getattr(self, key)

    def __setitem__(self, key, value):
        setattr(self, key, value)

    def __contains__(self, key):
        return key in self.__dict__

    @property
    def num_nodes(self) -> int:
        # PyG: no 'x' key, so num_nodes is inferred from node_attrs
        return int(self.node_attrs.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])

    def to(self, device, non_blocking: bool = False) -> "Data":
        out = self.__class__()
        for k, v in self.__dict__.items():
            if k.startswith("_eelg"):          # per-object caches (the model's CSR) stay behind
                continue
            setattr(out, k, v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v)
        return out


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list: List[Data], build_csr: bool = True) -> "Batch":
        b = cls()
        nn = [d.num_nodes for d in data_list]
        offs = np.concatenate([[0], np.cumsum(nn)])
        keys = data_list[0].keys()
        for k in keys:
            vals = [getattr(d, k) for d in data_list]
            if k == "edge_index":
                b.edge_index = torch.cat([v + int(o) for v, o in zip(vals, offs[:-1])], dim=1)
            elif k in _NODE_KEYS or k in _EDGE_KEYS:
                b[k] = torch.cat(vals, dim=0)
            elif k in _GRAPH_KEYS and torch.is_tensor(vals[0]):
                # per-graph targets: [1, 6, 6] / [1, 3, 3, 3, 3] / [6, 6] / scalar -> stacked
                b[k] = torch.cat([v if (v.dim() >= 3 and v.shape[0] == 1) else
                                  (v.unsqueeze(0) if v.dim() >= 1 else v.reshape(1)) for v in vals], dim=0)
            elif isinstance(vals[0], (int, float)) and not isinstance(vals[0], bool):
                b[k] = torch.tensor(vals)                   # PyG turns numbers into a [B] tensor
            elif torch.is_tensor(vals[0]):
                b[k] = torch.cat([v.reshape(1, *v.shape) for v in vals], dim=0)
            else:
                b[k] = vals
        b.batch = torch.repeat_interleave(torch.arange(len(data_list)), torch.tensor(nn))
        b.ptr = torch.from_numpy(offs.astype(np.int64))
        b.num_graphs = len(data_list)
        if build_csr:
            b.csr = build_edge_csr(b.edge_index, int(offs[-1]))
        return b


def collate(data_list: List[Data]) -> Batch:
    return Batch.from_data_list(data_list)


def morton_order(positions: torch.Tensor, bits: int = 10) -> torch.Tensor:
    """Node permutation along a Morton (Z-order) curve of the positions (quantised to
    ``bits`` per axis over the graph's bounding box): spatial neighbours get nearby ids."""
    pos = positions.detach().double().cpu()
    lo, hi = pos.min(0).values, pos.max(0).values
    scale = (1 << bits) - 1
    q = ((pos - lo) / (hi - lo).clamp_min(1e-12) * scale).long().clamp(0, scale)
    key = torch.zeros(pos.shape[0], dtype=torch.long)
    for bit in range(bits):
        for ax in range(3):
            key |= ((q[:, ax] >> bit) & 1) << (3 * bit + ax)
    return torch.argsort(key, stable=True)


def reorder_nodes(d: Data, perm: torch.Tensor) -> Data:
    """The same graph with node ``perm[i]`` renumbered ``i``: node tensors gathered, edge
    endpoints remapped, edges (and their shifts / radii) kept in order.  Graph-level outputs of
    the model are invariant (message passing is permutation-equivariant); the interaction
    kernels gather ``x[sender]`` from a smaller window of rows when neighbours have nearby ids
    (DESIGN.md section 6, config 5)."""
    import copy
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    e = copy.copy(d)
    for k in _NODE_KEYS:
        if k in d:
            e[k] = d[k][perm]
    e.edge_index = inv[d.edge_index]
    return e


def build_edge_csr(edge_index: torch.Tensor, num_nodes: int) -> Dict[str, torch.Tensor]:
    """Receiver-sorted edge order + CSR, and sender-CSR over that order.

    * ``perm``   [E] int64: ``edge_index[:, perm]`` is sorted by receiver (stable).
    * ``rowptr`` [N+1] int32: in-edges of node n are ``rowptr[n]:rowptr[n+1]``
      of the receiver-sorted order.
    * ``sperm``  [E] int32: positions (in the receiver-sorted order) of the edges,
      stably sorted by sender; ``srowptr`` [N+1] int32 is its CSR.
    Works on CPU or GPU tensors (torch ops only; no host round trip on GPU).
    """
    dev = edge_index.device
    snd, rcv = edge_index[0], edge_index[1]
    perm = torch.sort(rcv, stable=True).indices
    s_sorted = snd[perm]
    r_sorted = rcv[perm]
    # segment bounds of sorted keys by searchsorted: unlike bincount (which sizes its output
    # from the data) this never waits for the device
    bounds = torch.arange(num_nodes + 1, device=dev, dtype=r_sorted.dtype)
    rowptr = torch.searchsorted(r_sorted, bounds)
    sorted_s, sperm = torch.sort(s_sorted, stable=True)
    srowptr = torch.searchsorted(sorted_s, bounds)
    return {
        "perm": perm,
        "rowptr": rowptr.to(torch.int32),
        "sender": s_sorted.to(torch.int32).contiguous(),
        "receiver": r_sorted.to(torch.int32).contiguous(),
        "sperm": sperm.to(torch.int32).contiguous(),
        "srowptr": srowptr.to(torch.int32),
    }


def csr_to(csr: Dict[str, torch.Tensor], device) -> Dict[str, torch.Tensor]:
    return {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v)
            for k, v in csr.items()}


class DataLoader:
    """Tiny deterministic loader (shuffle with a seeded permutation)."""

    def __init__(self, dataset, batch_size: int, shuffle: bool = False, seed: int = 0,
                 indices: Optional[List[int]] = None):
        self.dataset, self.batch_size, self.shuffle, self.seed = dataset, batch_size, shuffle, seed
        self.indices = list(range(len(dataset))) if indices is None else list(indices)
        self.epoch = 0

    def __len__(self):
        return (len(self.indices) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        idx = self.indices
        if self.shuffle:
            g = np.random.default_rng(self.seed + self.epoch)
            idx = [idx[i] for i in g.permutation(len(idx))]
        self.epoch += 1
        for s in range(0, len(idx), self.batch_size):
            yield collate([self.dataset[i] for i in idx[s: s + self.batch_size]])
