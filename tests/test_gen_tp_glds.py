"""Host-side checks of the LDS-DMA tp_fwd generator (csrc/gen_kernels.py, no GPU needed).

The kernel moves one half-wave's rows for one edge as a static list of 16-byte chunks, 64
chunks per ``global_load_lds_dwordx4`` wave-instruction, and reads its operands back from the
lane-linear image at the float offsets the generator recorded.  For every generated TP set this
checks that the chunk list:
* covers, exactly once and in order, the group's weight slices of its channel group (first when
  ``TP_FWD_WNT``: the weight-only LDS-DMA instructions then carry the nontemporal policy), the
  x blocks of the group's l1 values (the channel group's part of each) and the whole padded SH
  row, for mul 16 / 32 / 64 (channel groups: mul = 64 two groups of 32, mul = 16 one of 16);
* has every source piece 16-byte aligned and inside its row (x: din, SH: the padded nshp,
  w: wn floats), so no LDS-DMA load leaves the tensors it reads;
* fits the image the kernel declares (ceil(chunks / 64) instructions of 64 chunks) and the
  image offsets the reads use point at the chunks holding those values;
and that the per-lane chunk descriptors, evaluated for every lane, reproduce the list.
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "energy-equiv-lattice-gnn_amd", "csrc")
sys.path.insert(0, CSRC)

import gen_kernels as gk  # noqa: E402
from gnn import cg  # noqa: E402

CONFIGS = gk.tp_configs()
MULS = gk.kernel_sets.MULS


def _setup(name, mul=32):
    saved, gk.MUL = gk.MUL, mul
    try:
        node, sh, target = gk.tp_configs()[name]
    finally:
        gk.MUL = saved
    paths = cg.tp_paths(node, sh, target)
    groups = gk._group_paths(sorted(paths, key=lambda p: (p.l1, p.l2, p.l3)), gk.TP_MAXACC)
    node_off = {ir.l: o for (m, ir), o in zip(node, node.offsets())}
    nshp = (sh.dim + 3) // 4 * 4
    wn = sum(p.mul for p in paths)
    return node, groups, node_off, nshp, wn


def _chunks(groups, nshp, node_off, mul, c):
    saved, gk.MUL = gk.MUL, mul
    try:
        return gk._glds_chunks(groups, nshp, node_off, 4, c)
    finally:
        gk.MUL = saved


@pytest.mark.parametrize("mul", MULS)
@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_chunk_lists_cover_the_rows_once_and_stay_in_bounds(name, mul):
    node, groups, node_off, nshp, wn = _setup(name, mul)
    din = node.dim
    n_cg, lw = max(1, mul // 32), min(mul, 32)
    seen = {0: set(), 2: set()}
    for c in range(n_cg):
        for (need_l1, need_l2, chunks, fo_x, fo_sh, fo_w), grp in zip(
                _chunks(groups, nshp, node_off, mul, c), groups):
            assert need_l1 == sorted({p.l1 for p in grp})
            expect = []

            def weights():
                for p in grp:
                    assert fo_w[p.slot] == 4 * len(expect)
                    expect.extend((2, 4 * (mul * p.slot + c * lw) + 16 * k) for k in range(lw // 4))
            if gk.TP_FWD_WNT:
                weights()
            for l in need_l1:
                assert fo_x[l] == 4 * len(expect)
                expect += [(0, 4 * (node_off[l] + c * lw * (2 * l + 1)) + 16 * k)
                           for k in range(lw * (2 * l + 1) // 4)]
            assert fo_sh == 4 * len(expect)
            expect += [(1, 16 * k) for k in range(nshp // 4)]
            if not gk.TP_FWD_WNT:
                weights()
            assert chunks == expect
            row_bytes = {0: 4 * din, 1: 4 * nshp, 2: 4 * wn}
            for kind, off in chunks:
                assert off % 16 == 0 and 0 <= off and off + 16 <= row_bytes[kind]
                if kind != 1:
                    seen[kind].add(off)
            assert len(set(chunks)) == len(chunks)
    # over all path groups and channel groups, every x block and weight slice is moved once
    assert len(seen[2]) == wn // 4
    assert len(seen[0]) == sum(mul * ir.dim for _, ir in node) // 4


def _eval_desc(line, lane):
    """evaluate one generated ``int kdJ, ofJ; { const int c_ = ...; kdJ = ...; ofJ = ...; }``"""
    m = re.match(r"\s*int kd(\d+), of\d+; \{ const int c_ = (\d+) \+ lane; kd\d+ = (.*); of\d+ = (.*); \}$", line)
    assert m, line
    j, base, kexpr, oexpr = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)
    c_ = base + lane

    def ev(e):
        # the expressions are nested (c_ < B ? A : REST) chains over integers
        e = e.strip()
        while e.startswith("(") and _matching(e, 0) == len(e) - 1:
            e = e[1:-1].strip()
        if "?" not in e:
            return eval(e, {}, {"c_": c_})          # noqa: S307  (generator arithmetic only)
        q = _top(e, "?")
        col = _top(e, ":", q)
        cond = eval(e[:q], {}, {"c_": c_})           # noqa: S307
        return ev(e[q + 1: col]) if cond else ev(e[col + 1:])
    return j, ev(kexpr), ev(oexpr)


def _matching(e, i):
    depth = 0
    for k in range(i, len(e)):
        depth += e[k] == "("
        depth -= e[k] == ")"
        if depth == 0:
            return k
    return -1


def _top(e, ch, start=0):
    depth = 0
    for k in range(start, len(e)):
        if e[k] == "(":
            depth += 1
        elif e[k] == ")":
            depth -= 1
        elif e[k] == ch and depth == 0:
            return k
    raise AssertionError(f"no top-level {ch!r} in {e}")


@pytest.mark.parametrize("name", ["tpA_l4", "tpB_l2", "tpB_l4"])
def test_lane_descriptors_reproduce_the_chunk_list(name):
    node, groups, node_off, nshp, wn = _setup(name)
    for need_l1, need_l2, chunks, fo_x, fo_sh, fo_w in gk._glds_chunks(groups, nshp, node_off):
        nj = -(-len(chunks) // 64)
        lines = gk._glds_desc(chunks, nj)
        assert len(lines) == nj
        for line in lines:
            for lane in range(64):
                j, kind, off = _eval_desc(line, lane)
                c = 64 * j + lane
                if c < len(chunks):
                    assert (kind, off) == chunks[c], (name, c)
                else:                                  # padding lanes: SH chunk 0 (in bounds)
                    assert (kind, off) == (1, 0)
