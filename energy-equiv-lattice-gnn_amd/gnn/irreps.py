"""Irreps bookkeeping for the product package (e3nn ``o3.Irreps`` semantics).

Only what the hot path needs: parse ``'32x0e+32x1o'``, repetition ``*``,
``sort`` (stable, natural parity first within one l), ``simplify``,
``count``, ``dim`` and block offsets.  Layout convention everywhere is e3nn's
mul-major-per-irrep row: block ``(mul, l)`` occupies ``mul*(2l+1)`` floats laid
out ``[mul][2l+1]``.
"""
from __future__ import annotations

from typing import Iterable, List, NamedTuple, Tuple


class Ir(NamedTuple):
    l: int
    p: int

    @staticmethod
    def parse(s) -> "Ir":
        if isinstance(s, Ir):
            return s
        if isinstance(s, tuple):
            return Ir(int(s[0]), int(s[1]))
        s = s.strip()
        l = int(s[:-1])
        return Ir(l, {"e": 1, "o": -1, "y": (-1) ** l}[s[-1]])

    @property
    def dim(self) -> int:
        return 2 * self.l + 1

    @property
    def natural(self) -> bool:
        return self.p == (-1) ** self.l

    def order_key(self):
        return (self.l, 0 if self.natural else 1)

    def times(self, other: "Ir") -> List["Ir"]:
        return [Ir(l, self.p * other.p) for l in range(abs(self.l - other.l), self.l + other.l + 1)]

    def __str__(self):
        return f"{self.l}{'e' if self.p == 1 else 'o'}"


class MulIr(NamedTuple):
    mul: int
    ir: Ir


class Irreps:
    def __init__(self, spec=None):
        if isinstance(spec, Irreps):
            self.items: Tuple[MulIr, ...] = spec.items
            return
        items: List[MulIr] = []
        if isinstance(spec, str):
            for term in filter(None, (t.strip() for t in spec.split("+"))):
                if "x" in term:
                    m, ir = term.split("x")
                    items.append(MulIr(int(m), Ir.parse(ir)))
                else:
                    items.append(MulIr(1, Ir.parse(term)))
        elif spec is not None:
            for it in spec:
                if isinstance(it, MulIr):
                    items.append(it)
                elif isinstance(it, (Ir, str)):
                    items.append(MulIr(1, Ir.parse(it)))
                else:
                    items.append(MulIr(int(it[0]), Ir.parse(it[1])))
        self.items = tuple(items)

    @staticmethod
    def spherical_harmonics(lmax: int) -> "Irreps":
        return Irreps([(1, Ir(l, (-1) ** l)) for l in range(lmax + 1)])

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]

    def __eq__(self, other):
        return isinstance(other, Irreps) and self.items == other.items

    def __add__(self, other):
        return Irreps(self.items + Irreps(other).items)

    def __mul__(self, n: int):
        return Irreps(self.items * n)

    def __contains__(self, ir) -> bool:
        ir = Ir.parse(ir)
        return any(x.ir == ir for x in self.items)

    @property
    def dim(self) -> int:
        return sum(m * ir.dim for m, ir in self.items)

    @property
    def num_irreps(self) -> int:
        return sum(m for m, _ in self.items)

    @property
    def lmax(self) -> int:
        return max(ir.l for _, ir in self.items)

    def count(self, ir) -> int:
        ir = Ir.parse(ir)
        return sum(m for m, x in self.items if x == ir)

    def offsets(self) -> List[int]:
        out, s = [], 0
        for m, ir in self.items:
            out.append(s)
            s += m * ir.dim
        return out

    def sort(self):
        """(sorted irreps, p) with p[old_index] = new_index (stable)."""
        order = sorted(range(len(self.items)), key=lambda i: (self.items[i].ir.order_key(), i))
        p = [0] * len(order)
        for new, old in enumerate(order):
            p[old] = new
        return Irreps([self.items[i] for i in order]), p

    def simplify(self) -> "Irreps":
        out: List[MulIr] = []
        for m, ir in self.items:
            if out and out[-1].ir == ir:
                out[-1] = MulIr(out[-1].mul + m, ir)
            elif m > 0:
                out.append(MulIr(m, ir))
        return Irreps(out)

    def __repr__(self):
        return "+".join(f"{m}x{ir}" for m, ir in self.items)

    __str__ = __repr__
