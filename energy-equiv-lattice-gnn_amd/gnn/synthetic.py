"""Synthetic periodic strut lattices with the reference's ``Data`` field layout.

The real GLAMM catalogue (``gnn/datasets.py:25-307``) needs an external
download and the empty ``lattices`` submodule, so benchmarks and tests use
this generator:

* graph g uses ``numpy.random.default_rng(seed + g)``;
* positions ~ U[0, a)^3 with ``a = 0.54 * N**(1/3)`` (mean nearest-neighbour
  distance ~0.3, inside the [0, 0.6] Gaussian range of ``gnn/model.py:147``);
* E/2 undirected struts: every node to its 2 nearest periodic (minimum-image)
  neighbours, de-duplicated, topped up with random near pairs to exactly E/2;
* each strut stored in both directions (``gnn/datasets.py:163-171``) with
  ``shifts = +-a * image`` so that ``pos[r] - pos[s] + shift`` is the strut
  vector (``gnn/mace.py:346``);
* ``edge_attr`` = strut radius ~ U[0.005, 0.05], equal for both directions
  (``gnn/datasets.py:198-199``); ``node_attrs`` = 1 (``:182``);
* ``stiffness`` = random SPD Mandel matrix ``A A^T / 6 + 0.1 I``.
"""
from __future__ import annotations

import numpy as np
import torch

from .data import Data


def _min_image(d: np.ndarray, a: float):
    img = -np.round(d / a)
    return d + img * a, img


def make_lattice(num_nodes: int, num_edges: int, seed: int) -> Data:
    assert num_edges % 2 == 0 and num_edges >= 2
    rng = np.random.default_rng(seed)
    n = num_nodes
    a = 0.54 * n ** (1.0 / 3.0)
    pos = rng.uniform(0.0, a, size=(n, 3))
    # the 8 nearest minimum-image neighbours of every node, in distance order (row blocks of
    # all-pairs distances; argpartition + sort of the 8 = the first 8 columns of a full argsort)
    kmax = min(n - 1, 8)
    order = np.empty((n, kmax), dtype=np.int64)
    if n > 2048:
        # large lattices (BASELINE config 5, ~5k nodes): periodic k-d tree, same neighbour set
        from scipy.spatial import cKDTree
        _, nb = cKDTree(pos, boxsize=a).query(pos, k=kmax + 1)
        for i in range(n):
            row = nb[i][nb[i] != i]
            order[i] = row[:kmax]
    for r0 in range(0, n if n <= 2048 else 0, 512):
        r1 = min(n, r0 + 512)
        d, _ = _min_image(pos[None, :, :] - pos[r0:r1, None, :], a)   # d[i, j] = pos[j] - pos[i]
        dist = np.linalg.norm(d, axis=-1)
        dist[np.arange(r1 - r0), np.arange(r0, r1)] = np.inf
        part = np.argpartition(dist, kmax - 1, axis=1)[:, :kmax]
        rows = np.arange(r1 - r0)[:, None]
        order[r0:r1] = part[rows, np.argsort(dist[rows, part], axis=1, kind="stable")]
    want = num_edges // 2
    pairs = {}
    for i in range(n):
        for j in order[i, :2]:
            key = (min(i, int(j)), max(i, int(j)))
            pairs.setdefault(key, None)
    # top up with random near pairs: i's 3rd..8th nearest neighbours, in random order
    cand = [(i, int(order[i, k])) for i in range(n) for k in range(2, kmax)]
    for t in rng.permutation(len(cand)):
        if len(pairs) >= want:
            break
        i, j = cand[t]
        pairs.setdefault((min(i, j), max(i, j)), None)
    keys = sorted(pairs.keys())
    assert len(keys) >= want, "lattice too small for the requested edge count"
    if len(keys) > want:
        sel = rng.choice(len(keys), size=want, replace=False)
        keys = [keys[t] for t in sorted(sel)]
    snd = np.array([p[0] for p in keys], dtype=np.int64)
    rcv = np.array([p[1] for p in keys], dtype=np.int64)
    _, image = _min_image(pos[rcv] - pos[snd], a)  # pos[r] - pos[s] + a*image = strut vector
    shifts = a * image
    radii = rng.uniform(0.005, 0.05, size=(want, 1))
    edge_index = np.stack([np.concatenate([snd, rcv]), np.concatenate([rcv, snd])])
    shifts = np.concatenate([shifts, -shifts], axis=0)
    radii = np.concatenate([radii, radii], axis=0)
    A = rng.normal(size=(6, 6))
    stiff = A @ A.T / 6.0 + 0.1 * np.eye(6)
    return Data(
        positions=torch.tensor(pos, dtype=torch.float32),
        node_attrs=torch.ones(n, 1, dtype=torch.float32),
        edge_index=torch.tensor(edge_index, dtype=torch.int64),
        shifts=torch.tensor(shifts, dtype=torch.float32),
        edge_attr=torch.tensor(radii, dtype=torch.float32),
        stiffness=torch.tensor(stiff, dtype=torch.float32).unsqueeze(0),
        rel_dens=torch.tensor([0.01], dtype=torch.float32),
        name=f"synthetic_{seed}",
    )


class SyntheticLattices:
    """Indexable dataset of ``count`` lattices; graph g uses seed ``seed + g``."""

    def __init__(self, count: int, num_nodes: int = 1024, num_edges: int = 4096, seed: int = 1234):
        self.count, self.num_nodes, self.num_edges, self.seed = count, num_nodes, num_edges, seed
        self._cache = {}

    def __len__(self):
        return self.count

    def __getitem__(self, g: int) -> Data:
        if g not in self._cache:
            self._cache[g] = make_lattice(self.num_nodes, self.num_edges, self.seed + g)
        return self._cache[g]

    @property
    def max_edge_radius(self) -> float:
        """``params.max_edge_radius = train_dset.data.edge_attr.max()`` (``scripts/train_main.py:64``)."""
        return float(max(self[g].edge_attr.max().item() for g in range(self.count)))
