"""Mandel <-> Cartesian rank-4 conversions with the convention of
``Cart_4_to_Mandel`` (``gnn/blocks.py:392-425``): Mandel index I -> (i, j) =
(0,0), (1,1), (2,2), (1,2), (0,2), (0,1); weights 1 for I < 3, sqrt(2) otherwise."""
import math

import torch

PAIRS = [(0, 0), (1, 1), (2, 2), (1, 2), (0, 2), (0, 1)]
W = [1.0, 1.0, 1.0, math.sqrt(2), math.sqrt(2), math.sqrt(2)]


def mandel_to_cart4(m: torch.Tensor) -> torch.Tensor:
    c = m.new_zeros(m.shape[:-2] + (3, 3, 3, 3))
    for a, (i, j) in enumerate(PAIRS):
        for b, (k, l) in enumerate(PAIRS):
            v = m[..., a, b] / (W[a] * W[b])
            for (p, q) in {(i, j), (j, i)}:
                for (r, s) in {(k, l), (l, k)}:
                    c[..., p, q, r, s] = v
    return c


def cart4_to_mandel(c: torch.Tensor) -> torch.Tensor:
    m = c.new_zeros(c.shape[:-4] + (6, 6))
    for a, (i, j) in enumerate(PAIRS):
        for b, (k, l) in enumerate(PAIRS):
            m[..., a, b] = W[a] * W[b] * c[..., i, j, k, l]
    return m


def rotate_mandel(m: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """``scripts/train_utils.py:122``: C'_abcd = Q_ai Q_bj Q_ck Q_dl C_ijkl."""
    c = mandel_to_cart4(m)
    c = torch.einsum("...ijkl,ai,bj,ck,dl->...abcd", c, q, q, q, q)
    return cart4_to_mandel(c)
