"""Lattice data path: catalogue entries -> ``Data`` -> rotation
augmentation -> Mandel targets, feeding the collate / CSR of ``gnn.data``.

Follows ``GLAMM_Dataset.process_one`` (``gnn/datasets.py:112-248``), ``RotateLat``
(``scripts/train_utils.py:114-146``) and the target scaling of ``load_datasets``
(``scripts/train_utils.py:204-239``).  The catalogue *file* reader
(``Catalogue.from_file``) and the helpers ``Lattice.calculate_transform_matrix``,
``Lattice.calculate_UC_volume`` and ``elasticity_func`` live in the un-vendored
``lattices`` submodule (empty in the reference checkout), so:

* entries are accepted as the dicts that ``Catalogue`` yields (the ``lat_data`` argument
  of ``process_one``: name, nodal_positions | reduced_node_coordinates,
  fundamental_edge_adjacency, fundamental_tesselation_vecs, lattice_constants,
  compliance_tensors_M | compliance_tensors_V, optional fundamental_edge_radii);
* the lattice transform, unit-cell volume and Voigt/Mandel/cartesian conversions are
  restated from their standard definitions (a, b, c, alpha, beta, gamma in degrees;
  Mandel order 11, 22, 33, 23, 13, 12 with sqrt(2) shear weights -- the order and
  weights of the model's own ``Cart_4_to_Mandel``, gnn/blocks.py:392-425, which the
  training loss compares against).  Parity of these three with ``lattices`` is
  unpinned (no source, no fixtures).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Iterable, List, Optional

import numpy as np
import torch

from .data import Data

# Mandel index of the symmetric index pair (i, j)
_PAIR = {(0, 0): 0, (1, 1): 1, (2, 2): 2, (1, 2): 3, (2, 1): 3, (0, 2): 4, (2, 0): 4,
         (0, 1): 5, (1, 0): 5}
_W = np.array([1.0, 1.0, 1.0, math.sqrt(2.0), math.sqrt(2.0), math.sqrt(2.0)])


def _mandel_maps():
    """[81] Mandel row/col and weight of every cartesian (ijkl)."""
    ij, kl, w = [], [], []
    for i in range(3):
        for j in range(3):
            for k in range(3):
                for l in range(3):
                    a, b = _PAIR[(i, j)], _PAIR[(k, l)]
                    ij.append(a)
                    kl.append(b)
                    w.append(_W[a] * _W[b])
    return np.array(ij), np.array(kl), np.array(w)


_IJ, _KL, _WW = _mandel_maps()


def cart4_to_mandel(c):
    """[..., 3, 3, 3, 3] (minor + major symmetric) -> [..., 6, 6] Mandel (numpy or torch)."""
    lib = torch if torch.is_tensor(c) else np
    flat = c.reshape(*c.shape[:-4], 81)
    out = lib.zeros((*c.shape[:-4], 6, 6), dtype=c.dtype) if lib is np else \
        torch.zeros((*c.shape[:-4], 6, 6), dtype=c.dtype, device=c.device)
    # every Mandel entry is hit by 1, 2 or 4 equal cartesian entries: take one of them
    first = {}
    for n in range(81):
        first.setdefault((_IJ[n], _KL[n]), n)
    for (a, b), n in first.items():
        out[..., a, b] = flat[..., n] * _WW[n]
    return out


def mandel_to_cart4(m):
    """[..., 6, 6] Mandel -> [..., 3, 3, 3, 3]."""
    if torch.is_tensor(m):
        ww = torch.tensor(_WW, dtype=m.dtype, device=m.device)
        flat = m[..., torch.as_tensor(_IJ, device=m.device), torch.as_tensor(_KL, device=m.device)] / ww
    else:
        flat = m[..., _IJ, _KL] / _WW
    return flat.reshape(*m.shape[:-2], 3, 3, 3, 3)


def voigt_to_mandel(v, kind: str):
    """Voigt 6x6 -> Mandel 6x6.  Stiffness: shear rows/cols x sqrt(2); compliance (engineering
    shear strains): shear rows/cols / sqrt(2)."""
    f = _W if kind == "stiffness" else 1.0 / _W
    if kind not in ("stiffness", "compliance"):
        raise ValueError(kind)
    fac = np.outer(f, f)
    return v * (torch.as_tensor(fac, dtype=v.dtype) if torch.is_tensor(v) else fac)


def mandel_to_voigt(m, kind: str):
    f = 1.0 / _W if kind == "stiffness" else _W
    if kind not in ("stiffness", "compliance"):
        raise ValueError(kind)
    fac = np.outer(f, f)
    return m * (torch.as_tensor(fac, dtype=m.dtype) if torch.is_tensor(m) else fac)


def transform_matrix(lattice_constants) -> np.ndarray:
    """Columns = lattice vectors for (a, b, c, alpha, beta, gamma[deg]) with a along x and b
    in the xy-plane: cartesian = reduced @ Q.T (gnn/datasets.py:158-160)."""
    a, b, c, al, be, ga = [float(v) for v in lattice_constants]
    al, be, ga = map(math.radians, (al, be, ga))
    cx = c * math.cos(be)
    cy = c * (math.cos(al) - math.cos(be) * math.cos(ga)) / math.sin(ga)
    cz = math.sqrt(max(c * c - cx * cx - cy * cy, 0.0))
    return np.array([[a, b * math.cos(ga), cx],
                     [0.0, b * math.sin(ga), cy],
                     [0.0, 0.0, cz]])


def unit_cell_volume(lattice_constants) -> float:
    a, b, c, al, be, ga = [float(v) for v in lattice_constants]
    ca, cb, cg = (math.cos(math.radians(t)) for t in (al, be, ga))
    return a * b * c * math.sqrt(max(1 - ca * ca - cb * cb - cg * cg + 2 * ca * cb * cg, 0.0))


def process_lattice(lat_data: Dict, edge_ft_format: str = "r", graph_ft_format: str = "cartesian_4",
                    reldens_slice: slice = slice(None), pre_filter: Optional[Callable] = None,
                    pre_transform: Optional[Callable] = None) -> List[Data]:
    """``GLAMM_Dataset.process_one`` (gnn/datasets.py:112-248): one ``Data`` per relative
    density of a catalogue entry."""
    name = lat_data["name"]
    if "nodal_positions" in lat_data:
        pos = np.atleast_2d(np.asarray(lat_data["nodal_positions"], dtype=float))
    elif "reduced_node_coordinates" in lat_data:
        pos = np.atleast_2d(np.asarray(lat_data["reduced_node_coordinates"], dtype=float))
    else:
        raise ValueError("No nodal positions found")
    adj = np.atleast_2d(np.asarray(lat_data["fundamental_edge_adjacency"], dtype=int))
    tess = np.atleast_2d(np.asarray(lat_data["fundamental_tesselation_vecs"], dtype=float))
    consts = np.asarray(lat_data["lattice_constants"], dtype=float)
    if "compliance_tensors_M" in lat_data:
        compl = dict(lat_data["compliance_tensors_M"])
    elif "compliance_tensors_V" in lat_data:
        compl = {k: (None if v is None else voigt_to_mandel(np.asarray(v, dtype=float), "compliance"))
                 for k, v in lat_data["compliance_tensors_V"].items()}
    else:
        compl = {}
    # keep the nodes that carry edges, renumbered densely
    uq = np.unique(adj)
    pos = pos[uq]
    adj = np.searchsorted(uq, adj)
    if tess.shape[1] == 6:
        tess = tess[:, 3:] - tess[:, :3]
    elif tess.shape[1] != 3:
        raise ValueError(f"Fundamental tessellation vectors shape {tess.shape} not recognised")
    unit_shifts = tess.astype(int)
    q = transform_matrix(consts)
    pos = pos @ q.T
    tess = tess @ q.T
    # both directions of every strut
    adj = np.vstack((adj, adj[:, ::-1]))
    unit_shifts = np.vstack((unit_shifts, -unit_shifts))
    tess = np.vstack((tess, -tess))
    evec = pos[adj[:, 1]] - pos[adj[:, 0]] + tess
    elen = np.linalg.norm(evec, axis=1)
    vol = unit_cell_volume(consts)
    n_nodes = len(np.unique(adj))
    common = dict(positions=torch.tensor(pos, dtype=torch.float32),
                  node_attrs=torch.ones((n_nodes, 1), dtype=torch.float32),
                  edge_index=torch.tensor(adj.T, dtype=torch.long),
                  shifts=torch.tensor(tess, dtype=torch.float32),
                  unit_shifts=torch.tensor(unit_shifts, dtype=torch.long))
    if not compl:
        raise AssertionError(f"Lattice {name} does not have enough data")
    out = []
    for rel_dens in list(compl.keys())[reldens_slice]:
        if "fundamental_edge_radii" in lat_data:
            radii_by_rd = lat_data["fundamental_edge_radii"]
            keys = list(radii_by_rd.keys())
            near = keys[int(np.argmin(np.abs(np.asarray(keys, dtype=float) - rel_dens)))]
            if abs(near - rel_dens) >= 1e-4:
                raise AssertionError(f"Closest relative density {near} is not close enough to {rel_dens}")
            r = np.asarray(radii_by_rd[near], dtype=float).reshape(-1, 1)
            radii = np.concatenate((r, r), axis=0)
            if radii.shape[0] != adj.shape[0]:
                raise AssertionError(f"Edge radii shape {radii.shape} does not match edge adjacency shape {adj.shape}")
        else:
            # uniform strut radius giving the requested relative density: rho V = pi r^2 sum L
            # (sum over both directions, as the reference)
            radii = math.sqrt(rel_dens * vol / (elen.sum() * math.pi)) * np.ones(adj.shape[0])
        comp = compl[rel_dens]
        stiff = None
        if comp is not None:
            comp = np.asarray(comp, dtype=float)
            stiff_m = np.linalg.inv(comp)
            if graph_ft_format == "Voigt":
                stiff = torch.from_numpy(mandel_to_voigt(stiff_m, "stiffness")).unsqueeze(0)
                comp = torch.from_numpy(mandel_to_voigt(comp, "compliance")).unsqueeze(0)
            elif graph_ft_format == "cartesian_4":
                stiff = torch.from_numpy(mandel_to_cart4(stiff_m)).unsqueeze(0)
                comp = torch.from_numpy(mandel_to_cart4(comp)).unsqueeze(0)
            elif graph_ft_format == "Mandel":
                stiff = torch.from_numpy(stiff_m).unsqueeze(0)
                comp = torch.from_numpy(comp).unsqueeze(0)
            else:
                raise ValueError(f"graph_ft_format {graph_ft_format!r}")
        cols = []
        for key in edge_ft_format.split(","):
            if key == "L":
                cols.append(elen.reshape(-1, 1))
            elif key == "r":
                cols.append(np.asarray(radii).reshape(-1, 1))
            elif key == "e_vec":
                cols.append(evec / elen.reshape(-1, 1))
            elif key == "euler":
                v = evec / elen.reshape(-1, 1)
                cols.append(np.column_stack((np.arccos(v[:, 2]), np.arctan2(v[:, 1], v[:, 0]) + np.pi)))
            else:
                raise ValueError(f"Unrecognised edge format string `{key}`")
        d = Data(name=name, **common, edge_attr=torch.tensor(np.column_stack(cols), dtype=torch.float32),
                 rel_dens=float(rel_dens), stiffness=stiff, compliance=comp)
        if pre_filter is not None and not pre_filter(d):
            continue
        if pre_transform is not None:
            d = pre_transform(d)
        out.append(d)
    return out


def rand_rotation(generator: Optional[torch.Generator] = None, dtype=torch.float32) -> torch.Tensor:
    """Uniform random proper rotation (QR of a Gaussian, sign-fixed, det +1)."""
    a = torch.randn(3, 3, generator=generator, dtype=torch.float64)
    q, r = torch.linalg.qr(a)
    q = q * torch.sign(torch.diagonal(r))
    if torch.det(q) < 0:
        q[:, 0] = -q[:, 0]
    return q.to(dtype)


class RotateLat:
    """``scripts/train_utils.py:114-146``: rotate positions, shifts and the cartesian
    stiffness / compliance by a random rotation (or ``Q``), then return Mandel targets."""

    def __init__(self, rotate: bool = True, generator: Optional[torch.Generator] = None):
        self.rotate = rotate
        self.generator = generator

    def __call__(self, lat: Data, Q: Optional[torch.Tensor] = None) -> Data:
        c, s, pos, shifts = lat.stiffness, lat.compliance, lat.positions, lat.shifts
        if self.rotate:
            if Q is None:
                Q = rand_rotation(self.generator)
            q = Q.to(c.dtype)
            c = torch.einsum("...ijkl,ai,bj,ck,dl->...abcd", c, q, q, q, q)
            s = torch.einsum("...ijkl,ai,bj,ck,dl->...abcd", s, q, q, q, q)
            pos = pos @ Q.to(pos.dtype).T
            shifts = shifts @ Q.to(shifts.dtype).T
        elif Q is not None:
            raise AssertionError("Q should be None if instance initialized with rotate=False")
        return Data(node_attrs=lat.node_attrs, edge_attr=lat.edge_attr, edge_index=lat.edge_index,
                    positions=pos, shifts=shifts, rel_dens=lat.rel_dens,
                    stiffness=cart4_to_mandel(c), compliance=cart4_to_mandel(s), name=lat.name)


class GLAMM_Dataset:  # noqa: N801
    """In-memory lattice dataset (``gnn/datasets.py:25-307``) over catalogue entries.

    ``entries`` are the per-lattice dicts of a catalogue (what ``lattices.Catalogue``
    yields); ``catalogue_path`` needs the un-vendored ``lattices`` package and raises.
    ``transform`` is applied on access, as in PyG's ``InMemoryDataset``."""

    def __init__(self, entries: Optional[Iterable[Dict]] = None, catalogue_path: Optional[str] = None,
                 edge_ft: str = "r", graph_ft_format: str = "cartesian_4", n_reldens: int = 1,
                 choose_reldens: str = "first", transform: Optional[Callable] = None,
                 pre_transform: Optional[Callable] = None, pre_filter: Optional[Callable] = None):
        if catalogue_path is not None:
            raise NotImplementedError(
                "reading .lat catalogue files needs the 'lattices' package (Catalogue.from_file), "
                "which is not vendored with the reference; pass the catalogue entries as dicts")
        slices = {"first": slice(None, n_reldens, 1), "last": slice(-n_reldens, None, 1),
                  "half": slice(None, 2 * n_reldens, 2), "all": slice(None, None, 1)}
        if choose_reldens not in slices:
            raise ValueError(f"choose_reldens `{choose_reldens}` not recognised")
        for key in edge_ft.split(","):
            if key not in ("L", "r", "e_vec", "euler"):
                raise ValueError(f"Edge feature format key `{key}` not recognised")
        self.transform = transform
        self.items: List[Data] = []
        for lat in entries or []:
            self.items.extend(process_lattice(lat, edge_ft, graph_ft_format, slices[choose_reldens],
                                              pre_filter, pre_transform))
        if not self.items:
            raise RuntimeError("Empty data list")

    def __len__(self) -> int:
        return len(self.items)

    def __getitem__(self, i: int) -> Data:
        d = self.items[i]
        return self.transform(d) if self.transform is not None else d

    def scale_targets(self, reldens_norm: bool = False) -> None:
        """``load_datasets`` scaling (scripts/train_utils.py:231-237): stiffness x 10/rel_dens
        (reldens_norm) or x 10000, compliance divided by the same factor."""
        for d in self.items:
            f = 10.0 / d.rel_dens if reldens_norm else 10000.0
            if d.stiffness is not None:
                d.stiffness = (d.stiffness * f).float()
                d.compliance = (d.compliance / f).float()
