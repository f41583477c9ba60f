#!/usr/bin/env python3
"""Build-time generator for the irreps-specialised HIP kernels (gfx950).

Emits ``generated/eelg_gen.hip``: straight-line, compile-time-indexed code for

* ``sh_eval_l<L>``           real spherical harmonics (recursion constants as literals)
* ``tp_fwd_<cfg>``           fused gather(x[sender]) -> 'uvu' CG tensor product ->
                             CSR segmented sum over in-edges -> / agg_norm_const
* ``tp_bwd_<cfg>``           per-edge grad of the TP weights and per-edge grad of
                             x[sender] (summed per sender by ``segment_sum_csr``)
* ``sc_fwd_<cfg>``           symmetric contraction as a sparse cubic polynomial
                             per (node, channel); coefficients are wave-uniform
                             (scalar loads), one wave = 64 nodes x 1 channel
* ``sc_bwd_x_<cfg>``         its gradient w.r.t. the node features
* ``sc_bwd_coef_<cfg>``      its gradient w.r.t. the per-term coefficients
                             (per-lane partial sums over nodes, LDS transpose-reduce)

Structure (CG sparsity, term lists, offsets) comes from ``gnn/cg.py``; the
C-ABI in ``eelg_capi.hip`` exposes each config by name together with a
structural hash that the Python host re-derives and checks at load time.
"""
from __future__ import annotations

import math
import os
import sys
from typing import Sequence, Dict, List, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from gnn import cg, kernel_sets  # noqa: E402
from gnn.irreps import Ir, Irreps  # noqa: E402

MUL = kernel_sets.MUL
# receivers per half-wave in tp_fwd (the launcher reads it from the config table)
TP_NPH = int(os.environ.get("EELG_TP_NPH", "8"))
TP_MAXACC = int(os.environ.get("EELG_TP_MAXACC", "64"))
TP_NOPIN_NEXT = int(os.environ.get("EELG_TP_NOPIN_NEXT", "0"))
TP_PIN_NEXT_LAST = int(os.environ.get("EELG_TP_PIN_NEXT_LAST", "1"))
TP_BWD_EPH = int(os.environ.get("EELG_TP_BWD_EPH", "1"))   # edges per half-wave in tp_bwd (4: 0.88 ms, 8: 0.90 ms vs 0.76 ms at 1)
TP_PK2 = int(os.environ.get("EELG_TP_PK2", "0"))        # packed channel-pair forward
TP_PK2_YNOW = int(os.environ.get("EELG_TP_PK2_YNOW", "0"))
TP_PK2_MAXACC = int(os.environ.get("EELG_TP_PK2_MAXACC", "16"))
TP_FOLDW = int(os.environ.get("EELG_TP_FOLDW", "1"))   # fold the path weight into x or y
TP_UNROLL2 = int(os.environ.get("EELG_TP_UNROLL2", "0"))
# symmetric contraction: nodes per lane.  2 = packed-fp32 v_pk_* arithmetic on node pairs;
# measured slower than 1 on MI355X (fwd 0.45 vs 0.35 ms, grad-x 0.76 vs 0.56, coef-grad 1.16 vs
# 0.86): twice the VGPRs and LDS per workgroup halve the occupancy, the SGPR coefficient
# operands need aligned pairs (s_mov per term), and dependent v_pk ops carry a wait state
SC_PK = int(os.environ.get("EELG_SC_PK", "1"))
# forward with two channels per lane (packed fp32: v_pk_mul / v_pk_fma with a channel-pair
# coefficient in one SGPR pair); the coefficients are then read channel-pair interleaved
SC_FWD_CP = int(os.environ.get("EELG_SC_FWD_CP", "0"))
SC_CP_MAXB = int(os.environ.get("EELG_SC_CP_MAXB", "16"))
# symmetric contraction: coefficient blocks (32 terms each) in flight ahead of the block being
# computed, forward / grad-x (r02: grad-x 0.56 -> 0.51 ms at 3; the forward spills SGPRs at 2+)
SC_PFD_FWD = int(os.environ.get("EELG_SC_PFD_FWD", "1"))
SC_PFD_BWD = int(os.environ.get("EELG_SC_PFD_BWD", "3"))
# symmetric contraction fwd / grad-x: 64-node tiles per workgroup (2: waves of one channel share
# its coefficient stream through the scalar cache; measured slower r03h: fwd 0.40 vs 0.37 ms)
SC_NT = int(os.environ.get("EELG_SC_NT", "1"))
# coefficient gradient: LDS-resident nodes per workgroup, waves per workgroup, sub-tile unroll
SC_COEF_CHUNK = int(os.environ.get("EELG_SC_COEF_CHUNK", "512"))
SC_COEF_WAVES = int(os.environ.get("EELG_SC_COEF_WAVES", "16"))
SC_COEF_UNROLL = int(os.environ.get("EELG_SC_COEF_UNROLL", "1"))
# nodes per lane per sweep step (2: operand pairs of adjacent nodes in one ds_read_b64, half the
# LDS read cycles per node) and the most accumulators (terms) per wave
SC_COEF_NPL = int(os.environ.get("EELG_SC_COEF_NPL", "1"))
SC_COEF_MAXJG = int(os.environ.get("EELG_SC_COEF_MAXJG", "64"))
# 1: the coefficient gradient reads the mul-major x / grad_out rows itself (no channel-major
# copies; grad-x 0.73 -> 0.57 ms but coef-grad 0.51 -> 0.58 ms, and the step measured 0.7 %
# slower, r02t); 0: it reads channel-major copies written by sc_bwd_x
SC_COEF_MULMAJOR = int(os.environ.get("EELG_SC_COEF_MULMAJOR", "0"))
TP_WPE = int(os.environ.get("EELG_TP_WPE", "0"))     # amdgpu_waves_per_eu floor for tp_fwd (0 = none)
# tp_fwd with the edge-uniform CG coupling M shared across channels through LDS (emit_tp_fwd_m)
# and its edge batch (phase-1 lanes per half-wave, a power of two <= 32)
TP_FWD_M = int(os.environ.get("EELG_TP_FWD_M", "0"))
TP_M_B = int(os.environ.get("EELG_TP_M_B", "8"))
TP_NOCOMPUTE = int(os.environ.get("EELG_TP_NOCOMPUTE", "0"))   # diagnostic only: tp_fwd without its CG arithmetic
TP_M_PAIR = int(os.environ.get("EELG_TP_M_PAIR", "0"))
# cooperative forward (emit_tp_fwd_coop): edges per tile per batch, receivers per tile, and the
# accumulator cap of its balanced path groups
TP_COOP = int(os.environ.get("EELG_TP_COOP", "0"))
TP_XCD_CONTIG = int(os.environ.get("EELG_TP_XCD_CONTIG", "1"))
TP_CO_BE = int(os.environ.get("EELG_TP_CO_BE", "4"))
TP_CO_R = int(os.environ.get("EELG_TP_CO_R", "16"))
TP_CO_MAXACC = int(os.environ.get("EELG_TP_CO_MAXACC", "36"))
TP_CO_WPE = int(os.environ.get("EELG_TP_CO_WPE", "0"))       # amdgpu_waves_per_eu floor (0 = none)
TP_M_AHEAD = int(os.environ.get("EELG_TP_M_AHEAD", "2"))      # coupling chunks read ahead of use


fnv1a64 = cg.fnv1a64


def flit(v: float) -> str:
    r = repr(float(v))
    if "e" not in r and "." not in r and "inf" not in r and "nan" not in r:
        r += ".0"
    return r + "f"


# ---------------------------------------------------------------------------
# configurations
# ---------------------------------------------------------------------------
def hidden_irreps(lmax: int, mul: int = MUL) -> Irreps:
    return Irreps("+".join(f"{mul}x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1)))


def tp_configs() -> Dict[str, Tuple[Irreps, Irreps, Irreps]]:
    """gnn/kernel_sets.py: node irreps 32x0e (tpA) or the hidden irreps (tpB) x SH(lmax)."""
    out = {}
    for lmax in kernel_sets.LMAX:
        sh = Irreps.spherical_harmonics(lmax)
        target = (sh * MUL).sort()[0].simplify()
        assert str(target) == kernel_sets.coupling_target(lmax)
        out[f"tpA_l{lmax}"] = (Irreps(f"{MUL}x0e"), sh, target)
        out[f"tpB_l{lmax}"] = (hidden_irreps(lmax), sh, target)
    return out


def sc_configs() -> Dict[str, Tuple[str, Tuple[int, ...], int]]:
    """coupling = the interaction irreps (SH lmax), outputs = the hidden irreps, correlation
    1..3 (gnn/kernel_sets.py).  Hidden irreps beyond the SH lmax are not generated: the
    reference's U_matrix_real fails for them (an output irrep with no degree-1 path leaves
    ``last_ir`` unbound, gnn/mace.py:466-476)."""
    out = {}
    for lmax in kernel_sets.LMAX:
        for corr in kernel_sets.CORRELATIONS:
            out[f"sc_l{lmax}_c{corr}"] = (kernel_sets.coupling_str(lmax), tuple(range(lmax + 1)), corr)
    return out


tp_signature = cg.tp_signature
sc_signature = cg.sc_signature


# ---------------------------------------------------------------------------
# spherical harmonics
# ---------------------------------------------------------------------------
def emit_sh(lmax: int) -> str:
    L = []
    L.append(f"// real SH up to l={lmax}, e3nn 'component' normalisation, input need not be unit")
    L.append(f"__device__ __forceinline__ void sh_eval_l{lmax}(float vx, float vy, float vz, float* __restrict__ out) {{")
    L.append("  float n = sqrtf(vx * vx + vy * vy + vz * vz);")
    L.append("  float inv = 1.0f / fmaxf(n, 1e-12f);")
    L.append("  float v0 = vx * inv, v1 = vy * inv, v2 = vz * inv;")
    L.append("  float y0_0 = 1.0f;")
    if lmax >= 1:
        L.append("  float y1_0 = v0, y1_1 = v1, y1_2 = v2;")
    for l, terms in enumerate(cg.sh_recursion(lmax), start=1):
        acc: Dict[int, List[str]] = {}
        for i, j, k, c in terms:
            acc.setdefault(k, []).append(f"{flit(c)} * y{l}_{i} * v{j}")
        for k in range(2 * l + 3):
            expr = " + ".join(acc.get(k, ["0.0f"]))
            L.append(f"  float y{l + 1}_{k} = {expr};")
    idx = 0
    for l in range(lmax + 1):
        s = math.sqrt(2 * l + 1)
        for m in range(2 * l + 1):
            L.append(f"  out[{idx}] = {flit(s)} * y{l}_{m};")
            idx += 1
    L.append("}")
    return "\n".join(L)


# ---------------------------------------------------------------------------
# tensor product
# ---------------------------------------------------------------------------
def _path_cg(p: cg.TPPath):
    return cg.nonzeros(cg.wigner_3j(p.l1, p.l2, p.l3))


def _group_paths(paths: List[cg.TPPath], max_acc: int) -> List[List[cg.TPPath]]:
    """Contiguous groups (slot order) with <= max_acc accumulators per lane."""
    groups, cur, n = [], [], 0
    for p in paths:
        d = 2 * p.l3 + 1
        if cur and n + d > max_acc:
            groups.append(cur)
            cur, n = [], 0
        cur.append(p)
        n += d
    if cur:
        groups.append(cur)
    return groups


def _emit_t(p: cg.TPPath, xname, yname, tname, L: List[str], ind: str):
    """t_k = sum_{ij} C_ijk x_i y_j for one path; picks the cheaper of
    pair-products-first and M-first (M_ik = sum_j C_ijk y_j)."""
    nz = _path_cg(p)
    pairs = sorted({(i, j) for (i, j, k), _ in nz})
    iks = sorted({(i, k) for (i, j, k), _ in nz})
    d3 = 2 * p.l3 + 1
    terms_by_k: Dict[int, List] = {k: [] for k in range(d3)}
    if len(pairs) <= len(iks):
        for i, j in pairs:
            L.append(f"{ind}const float z{i}_{j} = {xname(p, i)} * {yname(p, j)};")
        for (i, j, k), c in nz:
            terms_by_k[k].append(f"{flit(c)} * z{i}_{j}")
    else:
        byik: Dict[Tuple[int, int], List[str]] = {}
        for (i, j, k), c in nz:
            byik.setdefault((i, k), []).append(f"{flit(c)} * {yname(p, j)}")
        for (i, k), ts in byik.items():
            L.append(f"{ind}const float m{i}_{k} = {' + '.join(ts)};")
            terms_by_k[k].append(f"{xname(p, i)} * m{i}_{k}")
    for k in range(d3):
        expr = " + ".join(terms_by_k[k]) if terms_by_k[k] else "0.0f"
        L.append(f"{ind}const float {tname}{k} = {expr};")


def _emit_acc(p: cg.TPPath, xname, yname, aname, L: List[str], ind: str):
    """a_k += sum_{ij} C_ijk x_i y_j for one path, straight into the accumulators (the path
    weight already folded into x or y); cheaper of pair-products-first and M-first."""
    nz = _path_cg(p)
    pairs = sorted({(i, j) for (i, j, k), _ in nz})
    iks = sorted({(i, k) for (i, j, k), _ in nz})
    if len(pairs) <= len(iks):
        # each pair product is followed by the terms using it (short live ranges)
        byij: Dict[Tuple[int, int], List] = {}
        for (i, j, k), c in nz:
            byij.setdefault((i, j), []).append((k, c))
        for i, j in pairs:
            L.append(f"{ind}{{ const float z = {xname(p, i)} * {yname(p, j)};")
            for k, c in byij[(i, j)]:
                L.append(f"{ind}  {aname(k)} = fmaf({flit(c)}, z, {aname(k)});")
            L.append(f"{ind}}}")
    else:
        byik: Dict[Tuple[int, int], List[str]] = {}
        for (i, j, k), c in nz:
            byik.setdefault((i, k), []).append(f"{flit(c)} * {yname(p, j)}")
        for (i, k), ts in byik.items():
            L.append(f"{ind}{aname(k)} = fmaf({xname(p, i)}, {' + '.join(ts)}, {aname(k)});")


_VT = {4: "eelg_f4u", 3: "eelg_f3u", 2: "eelg_f2u"}


def vec_load(names: Sequence[str], base: str, start: str) -> List[str]:
    """names[i] = base[start + i] with dword-aligned 4/3/2-wide loads (start is an expr)."""
    out, i = [], 0
    while i < len(names):
        w = min(4, len(names) - i)
        if w == 1:
            out.append(f"{names[i]} = {base}[{start} + {i}];")
        else:
            out.append(f"{{ const {_VT[w]} v_ = *reinterpret_cast<const {_VT[w]}*>({base} + {start} + {i}); "
                       + " ".join(f"{names[i + k]} = v_[{k}];" for k in range(w)) + " }")
        i += w
    return out


def vec_store(vals: Sequence[str], base: str, start: str) -> List[str]:
    out, i = [], 0
    while i < len(vals):
        w = min(4, len(vals) - i)
        if w == 1:
            out.append(f"{base}[{start} + {i}] = {vals[i]};")
        else:
            out.append(f"*reinterpret_cast<{_VT[w]}*>({base} + {start} + {i}) = {_VT[w]}{{"
                       + ", ".join(vals[i: i + w]) + "};")
        i += w
    return out


def sh_load(need_l2: Sequence[int], pref: str, base: str) -> List[str]:
    """The needed SH components from a 16-B aligned padded row: one float4 per fully needed
    16-B block, narrower loads of exactly the needed runs otherwise.  (A float4 whose lanes are
    partly unused would leave destination registers the compiler may reuse while the load is
    in flight, which forces a wait for it: the last row block holds y24 alone at lmax 4.)"""
    need = sorted({l * l + j for l in need_l2 for j in range(2 * l + 1)})
    out = []
    for b in sorted({j // 4 for j in need}):
        comps = [j for j in need if j // 4 == b]
        if len(comps) == 4:
            out.append(f"{{ const eelg_f4a v_ = *reinterpret_cast<const eelg_f4a*>({base} + {4 * b}); "
                       + " ".join(f"{pref}y{j} = v_[{j - 4 * b}];" for j in comps) + " }")
            continue
        runs, cur = [], [comps[0]]
        for j in comps[1:]:
            if j == cur[-1] + 1:
                cur.append(j)
            else:
                runs.append(cur)
                cur = [j]
        runs.append(cur)
        for r in runs:
            out += vec_load([f"{pref}y{j}" for j in r], base, str(r[0]))
    return out


def emit_tp_fwd_pk2(name, sfx, WT, bf, groups, din, nshp, wn, dmid, node_off) -> List[str]:
    """Packed-fp32 forward (TP_PK2): a lane owns the channel PAIR (c0, c0 + 1) of one
    receiver stream, 16 lanes per stream, 4 streams per wave.  The CG contractions run in
    M-first form: M_ik = sum_j C_ijk y_j is edge-only data (scalar VALU with literal CG
    constants, shared by the two channels) and a_k += (w x_i) M_ik is one v_pk_fma_f32 for
    both channels; the path weight is folded into the x pair."""
    L: List[str] = []
    ng = len(groups)
    wpe = f" __attribute__((amdgpu_waves_per_eu({TP_WPE})))" if TP_WPE else ""
    L.append(f"__global__ __launch_bounds__(256){wpe} void tp_fwd_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ rowptr, int n_nodes,")
    L.append("    float inv_norm, float* __restrict__ agg) {")
    L.append("  const int lane = threadIdx.x & 63;")
    L.append("  const int c0 = (lane & 15) * 2;")
    L.append(f"  const int q = blockIdx.x >> 3, grp = q % {ng};")
    if TP_XCD_CONTIG:
        # XCD k (blockIdx % 8) takes one contiguous range of node tiles, walked in order: the
        # x rows of a lattice are gathered by one XCD (its L2) rather than by all eight
        L.append(f"  const int ntl = (n_nodes + {8 * TP_NPH - 1}) / {8 * TP_NPH}, tpx = (ntl + 7) >> 3;")
        L.append(f"  const int tile = (blockIdx.x & 7) * tpx + q / {ng};")
    else:
        L.append(f"  const int tile = (q / {ng}) * 8 + (blockIdx.x & 7);")
    L.append(f"  const int n0 = ((tile * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4)) * {TP_NPH};")
    L.append("  if (n0 >= n_nodes) return;")
    L.append(f"  const int n1 = min(n0 + {TP_NPH}, n_nodes);")
    L.append("  switch (grp) {")
    for gi, grp in enumerate(groups):
        L.append(f"  case {gi}: {{")
        need_l1 = sorted({p.l1 for p in grp})
        need_l2 = sorted({p.l2 for p in grp})
        accs = [f"a{p.slot}_{k}" for p in grp for k in range(2 * p.l3 + 1)]
        L.append("    eelg_f2 " + ", ".join(f"{a} = {{0.0f, 0.0f}}" for a in accs) + ";")
        ysh = [f"y{l * l + j}" for l in need_l2 for j in range(2 * l + 1)]
        curf = ([f"xr{l}_{i}" for l in need_l1 for i in range(2 * (2 * l + 1))]
                + ([] if TP_PK2_YNOW else ysh))
        curv = [f"w{p.slot}" for p in grp]

        def load(pref, ev, sv, guard):
            out = [f"    {{ const bool ok = {guard};",
                   f"      const float* __restrict__ xs = x + (size_t){sv} * {din};",
                   f"      const float* __restrict__ ye = sh + (size_t)(ok ? {ev} : 0) * {nshp};",
                   f"      const {WT}* __restrict__ we = w + (size_t)(ok ? {ev} : 0) * {wn} + c0;"]
            for l in need_l1:
                d = 2 * l + 1
                # channels c0, c0 + 1 of block l: 2d consecutive floats
                out += ["      " + ln for ln in vec_load([f"{pref}xr{l}_{i}" for i in range(2 * d)], "xs",
                                                          f"{node_off[l]} + c0 * {d}")]
            if not TP_PK2_YNOW:
                out += ["      " + ln for ln in sh_load(need_l2, pref, "ye")]
            for p in grp:
                if bf:
                    out.append(f"      {{ const unsigned v_ = *reinterpret_cast<const unsigned*>(we + {p.slot * MUL}); "
                               f"{pref}w{p.slot} = eelg_f2{{__uint_as_float(v_ << 16), __uint_as_float(v_ & 0xffff0000u)}}; }}")
                else:
                    out.append(f"      {pref}w{p.slot} = *reinterpret_cast<const eelg_f2*>(we + {p.slot * MUL});")
            out.append("    }")
            return out
        L.append("    int e = rowptr[n0];")
        L.append("    const int eend = rowptr[n1];")
        L.append("    int node = n0, nend = rowptr[n0 + 1], nend2 = rowptr[min(n0 + 2, n1)];")
        L.append("    int s1 = e + 1 < eend ? sender[e + 1] : 0;")
        L.append("    float " + ", ".join(curf) + ";")
        L.append("    eelg_f2 " + ", ".join(curv) + ";")
        L += load("", "e", "(e < eend ? sender[e] : 0)", "e < eend")
        cur = curf + curv
        L.append("    for (;;) {")
        L.append("      float " + ", ".join("n" + v for v in curf) + ";")
        L.append("      eelg_f2 " + ", ".join("n" + v for v in curv) + ";")
        L.append("      while (node < n1 && nend == e) {")
        L.append(f"        float* __restrict__ o = agg + (size_t)node * {dmid};")
        for p in grp:
            d3 = 2 * p.l3 + 1
            vals = [f"a{p.slot}_{k}.x" for k in range(d3)] + [f"a{p.slot}_{k}.y" for k in range(d3)]
            L.extend("        " + ln for ln in vec_store(vals, "o", f"{p.out_off} + c0 * {d3}"))
        L.append("        " + " ".join(f"{a} = eelg_f2{{0.0f, 0.0f}};" for a in accs))
        L.append("        ++node; nend = nend2; nend2 = rowptr[min(node + 2, n1)];")
        L.append("      }")
        L.append("      if (e >= eend) break;")
        L.append("      { const int s2 = e + 2 < eend ? sender[e + 2] : 0;")
        if TP_PK2_YNOW:
            # this edge's SH row, loaded now (no prefetch registers for it)
            L.append("        float " + ", ".join(ysh) + ";")
            L.append(f"        {{ const float* __restrict__ ye = sh + (size_t)e * {nshp};")
            L += ["          " + ln for ln in sh_load(need_l2, "", "ye")]
            L.append("        }")
        L.extend("  " + ln for ln in load("n", "e + 1", "s1", "e + 1 < eend"))
        cpin_mid = pin(accs + cur)
        cpin_last = pin(accs + cur + ["n" + v for v in cur])
        for p in grp:
            d1 = 2 * p.l1 + 1
            L.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
            L.append(f"        const eelg_f2 wp = w{p.slot} * ({flit(p.coef)} * inv_norm);")
            for i in range(d1):
                L.append(f"        const eelg_f2 xw{i} = eelg_f2{{xr{p.l1}_{i}, xr{p.l1}_{d1 + i}}} * wp;")
            nz = _path_cg(p)
            byik: Dict[Tuple[int, int], List[str]] = {}
            for (i, j, k), c in nz:
                byik.setdefault((i, k), []).append(f"{flit(c)} * y{p.l2 * p.l2 + j}")
            for (i, k), ts in byik.items():
                L.append(f"        {{ const float m = {' + '.join(ts)}; "
                         f"a{p.slot}_{k} = eelg_fma2(xw{i}, eelg_f2{{m, m}}, a{p.slot}_{k}); }}")
            L.append("      }")
            L.append("      " + (cpin_last if p is grp[-1] else cpin_mid))
        L.append("      s1 = s2; ++e; }")
        L.append("      " + " ".join(f"{v} = n{v};" for v in cur))
        L.append("    }")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    return L


def _group_entries(grp: List[cg.TPPath]):
    """The edge-uniform coupling entries of a path group: for every path p and nonzero (i, k)
    of its CG block, M_p[i, k] = sum_j coef_p * C_ijk * y_j (the path normalisation folded in).
    Returns [(p, i, k, [(c, j), ...])] in path order; within a path (i, k) order when the path
    weight is folded into x (d1 <= d3), (k, i) order when it is applied to the path result, so
    the forward consumes the entries strictly in order (few chunks live at a time)."""
    ents = []
    for p in grp:
        by: Dict[Tuple[int, int], List[Tuple[float, int]]] = {}
        for (i, j, k), c in _path_cg(p):
            by.setdefault((i, k), []).append((c * p.coef, p.l2 * p.l2 + j))
        key = (lambda ik: ik) if 2 * p.l1 + 1 <= 2 * p.l3 + 1 else (lambda ik: (ik[1], ik[0]))
        for (i, k) in sorted(by, key=key):
            ents.append((p, i, k, by[(i, k)]))
    return ents


def emit_tp_fwd_m(name, sfx, WT, ld_w, groups, din, nshp, nsh, wn, dmid, node_off) -> List[str]:
    """Forward with the edge-uniform CG coupling shared across the channels through LDS.

    For an edge, every channel u of path p computes out_k += w_p[u] * sum_i M_p[i,k] x_i[u]
    with M_p[i,k] = sum_j coef_p C_ijk y_j: M depends on the edge only, so the per-channel
    form (what the straight-line per-lane code evaluates redundantly in all 32 lanes) costs
    nnz + (i,k) products per lane, while with M given it costs one FMA per (i,k).

    * Phase 1, every TP_M_B edges: lane s (= lane & (B-1)) of a half-wave evaluates the
      group's M entries for edge e + s of its stream (straight-line, literal CG constants,
      inv_norm folded into y) and stores them to the half-wave's LDS slab in chunk-major
      float4s [chunk][slot][4] (B lanes write B consecutive float4: conflict-free).  The SH
      rows of the next batch are loaded meanwhile (one row per lane, a batch ahead).
    * Phase 2, per edge: the 32 lanes (= channels) read the edge's chunks as broadcast
      ds_read_b128 and apply them to x[sender] with the path weight folded into the shorter
      of x (d1) or the path result (d3).
    * TP_M_PAIR: two edges per loop iteration, whose x[sender] / w rows are loaded together
      one iteration ahead (sender indices two iterations ahead): two edges' loads in flight
      per wave at every wait instead of one (the copy of the prefetched registers at the end
      of an iteration is where the wave waits for them).
    The receiver-segmented sum, flush and XCD placement are tp_fwd's.  Every iteration but a
    stream's last consumes the same number of edges in both half-waves, so the batch boundary
    is uniform across the wave."""
    B = TP_M_B
    PAIR = TP_M_PAIR
    assert B >= 2 and B & (B - 1) == 0
    ng = len(groups)
    gents = [_group_entries(g) for g in groups]
    maxch = max((len(e) + 3) // 4 for e in gents)
    slab = maxch * B + 1                       # float4s per half-wave (+1: bank offset between halves)
    L: List[str] = []
    L.append(f"__global__ __launch_bounds__(256) void tp_fwd_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ rowptr, int n_nodes,")
    L.append("    float inv_norm, float* __restrict__ agg) {")
    L.append(f"  __shared__ float4 mbuf[8 * {slab}];")
    L.append("  const int lane = threadIdx.x & 63;")
    L.append(f"  const int u = lane & {MUL - 1};")
    L.append(f"  const int slot = lane & {B - 1};")
    L.append(f"  const bool writer = (lane & 31) < {B};")
    L.append(f"  float4* __restrict__ mb = mbuf + (threadIdx.x >> 5) * {slab};")
    L.append(f"  const int q = blockIdx.x >> 3, grp = q % {ng};")
    if TP_XCD_CONTIG:
        # XCD k (blockIdx % 8) takes one contiguous range of node tiles, walked in order: the
        # x rows of a lattice are gathered by one XCD (its L2) rather than by all eight
        L.append(f"  const int ntl = (n_nodes + {8 * TP_NPH - 1}) / {8 * TP_NPH}, tpx = (ntl + 7) >> 3;")
        L.append(f"  const int tile = (blockIdx.x & 7) * tpx + q / {ng};")
    else:
        L.append(f"  const int tile = (q / {ng}) * 8 + (blockIdx.x & 7);")
    L.append(f"  const int n0 = ((tile * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5)) * {TP_NPH};")
    L.append("  if (n0 >= n_nodes) return;")
    L.append(f"  const int n1 = min(n0 + {TP_NPH}, n_nodes);")
    L.append("  switch (grp) {")
    only = os.environ.get("EELG_TP_M_ONLY")            # register-budget probe: one group only
    for gi, (grp, ents) in enumerate(zip(groups, gents)):
        if only is not None and gi != int(only):
            continue
        L.append(f"  case {gi}: {{")
        need_l1 = sorted({p.l1 for p in grp})
        need_j = sorted({j for *_, ts in ents for _, j in ts})
        need_l2 = sorted({l for l in range(9) for j in need_j if l * l <= j < (l + 1) * (l + 1)})
        accs = [f"a{p.slot}_{k}" for p in grp for k in range(2 * p.l3 + 1)]
        xw_ = [f"x{l}_{i}" for l in need_l1 for i in range(2 * l + 1)] + [f"w{p.slot}" for p in grp]
        ys_ = [f"y{l * l + j}" for l in need_l2 for j in range(2 * l + 1)]
        nch = (len(ents) + 3) // 4
        sets = ["c0_", "c1_"] if PAIR else ["c0_"]        # register sets in use (one per edge)
        nsets = ["n0_", "n1_"] if PAIR else ["n0_"]       # their prefetch
        L.append("    float " + ", ".join(f"{a} = 0.0f" for a in accs) + ";")
        L.append("    int e = rowptr[n0];")
        L.append("    const int eend = rowptr[n1];")
        L.append("    int node = n0, nend = rowptr[n0 + 1], nend2 = rowptr[min(n0 + 2, n1)];")
        L.append("    float " + ", ".join(pf + v for pf in sets for v in xw_) + ", " + ", ".join(ys_) + ";")

        def ld_xw(pref, ev, sv, ind="    "):
            """x[sender] slices and the group's weights of edge ``ev`` (clamped addresses when
            the edge does not exist: the values are then never used)"""
            out = [f"{ind}{{ const bool ok = {ev} < eend;",
                   f"{ind}  const float* __restrict__ xs = x + (size_t)(ok ? {sv} : 0) * {din};",
                   f"{ind}  const {WT}* __restrict__ we = w + (size_t)(ok ? {ev} : 0) * {wn} + u;"]
            for l in need_l1:
                d = 2 * l + 1
                out += [f"{ind}  " + ln for ln in vec_load([f"{pref}x{l}_{i}" for i in range(d)], "xs",
                                                          f"{node_off[l]} + u * {d}")]
            for p in grp:
                out.append(f"{ind}  {pref}w{p.slot} = {ld_w(f'we[{p.slot * MUL}]')};")
            out.append(f"{ind}}}")
            return out

        def ld_y(ev, ind="    "):
            """this lane's SH row of edge ``ev`` straight into the y registers (clamped; rows
            past the stream are unused); consumed by the next phase 1, a batch later"""
            out = [f"{ind}{{ const float* __restrict__ ye = sh + (size_t)min({ev}, max(eend - 1, 0)) * {nshp};"]
            out += [f"{ind}  " + ln for ln in sh_load(need_l2, "", "ye")]
            out.append(f"{ind}}}")
            return out

        def flush(ind):
            out = [f"{ind}while (node < n1 && nend == e) {{",
                   f"{ind}  float* __restrict__ o = agg + (size_t)node * {dmid};"]
            for p in grp:
                d3 = 2 * p.l3 + 1
                out.extend(f"{ind}  " + ln for ln in vec_store([f"a{p.slot}_{k}" for k in range(d3)], "o",
                                                              f"{p.out_off} + u * {d3}"))
            out.append(f"{ind}  " + " ".join(f"{a} = 0.0f;" for a in accs))
            out.append(f"{ind}  ++node; nend = nend2; nend2 = rowptr[min(node + 2, n1)];")
            out.append(f"{ind}}}")
            return out

        # phase 2 consumes the entries in order; chunk c + TP_M_AHEAD is read when chunk c is
        # first used, and a pin with a memory clobber after each chunk keeps the reads there
        # (the compiler would otherwise hoist every chunk read: registers)
        AH = TP_M_AHEAD

        def compute(cp, es, ind):
            out = [f"{ind}{{"]
            loaded = set()
            state = {"cur": -1}
            pn = pin(accs + [pf + v for pf in sets for v in xw_], memory=True)

            def need(t):
                c = t // 4
                if c != state["cur"]:
                    if state["cur"] >= 0:
                        out.append(f"{ind}" + pn)
                    for cc in range(c, min(c + AH + 1, nch)):
                        if cc not in loaded:
                            loaded.add(cc)
                            out.append(f"{ind}const float4 mc{cc} = mb[{cc * B} + {es}];")
                    state["cur"] = c
                return f"mc{c}.{'xyzw'[t % 4]}"
            t = 0
            for p in grp:
                d1, d3 = 2 * p.l1 + 1, 2 * p.l3 + 1
                pents = [e_ for e_ in ents if e_[0] is p]
                out.append(f"{ind}// slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}, {len(pents)} coupling entries")
                if d1 <= d3:
                    for i in range(d1):
                        out.append(f"{ind}const float xw{p.slot}_{i} = {cp}x{p.l1}_{i} * {cp}w{p.slot};")
                    for e_ in pents:
                        _, i, k, _ = e_
                        m = need(t)
                        out.append(f"{ind}a{p.slot}_{k} = fmaf({m}, xw{p.slot}_{i}, a{p.slot}_{k});")
                        t += 1
                else:
                    n = 0
                    while n < len(pents):
                        k = pents[n][2]
                        run = []
                        while n < len(pents) and pents[n][2] == k:
                            run.append(pents[n])
                            n += 1
                        m = need(t)
                        out.append(f"{ind}float t{p.slot}_{k} = {m} * {cp}x{p.l1}_{run[0][1]};")
                        t += 1
                        for e_ in run[1:]:
                            m = need(t)
                            out.append(f"{ind}t{p.slot}_{k} = fmaf({m}, {cp}x{p.l1}_{e_[1]}, t{p.slot}_{k});")
                            t += 1
                        out.append(f"{ind}a{p.slot}_{k} = fmaf({cp}w{p.slot}, t{p.slot}_{k}, a{p.slot}_{k});")
            out.append(f"{ind}" + pn)
            out.append(f"{ind}}}")
            return out

        # prologue: this batch's SH rows, the first edges' operands, sender indices ahead
        L += ld_y("e + slot")
        for k, pf in enumerate(sets):
            L += ld_xw(pf, f"e + {k}", f"sender[e + {k}]")
        nxt = len(sets)
        L.append("    " + " ".join(f"int s{k} = sender[min(e + {nxt + k}, max(eend - 1, 0))];"
                                   for k in range(len(sets))))
        L.append("    const int ebase = e;")
        L.append("    for (;;) {")
        L.append("      float " + ", ".join(pf + v for pf in nsets for v in xw_) + ";")
        L += flush("      ")
        L.append("      if (e >= eend) break;")
        # ---- phase 1 at a batch boundary: M of edges e .. e+B-1 into the slab ----
        L.append(f"      if (((e - ebase) & {B - 1}) == 0) {{")
        L.append("        " + " ".join(f"y{j} *= inv_norm;" for j in need_j))
        for c in range(nch):
            vals = []
            for t in range(4 * c, 4 * c + 4):
                if t >= len(ents):
                    vals.append("0.0f")
                    continue
                _, _, _, ts = ents[t]
                ex = f"{flit(ts[0][0])} * y{ts[0][1]}"
                for cc, j in ts[1:]:
                    ex = f"fmaf({flit(cc)}, y{j}, {ex})"
                vals.append(ex)
            L.append(f"        {{ const float4 m_ = make_float4({', '.join(vals)});")
            L.append(f"          if (writer) mb[{c * B} + slot] = m_; }}")
            # each chunk is computed and stored in place (not hoisted: registers)
            L.append("        " + pin([f"y{j}" for j in need_j], memory=True))
        L.append("        __builtin_amdgcn_wave_barrier();")
        L += ld_y(f"e + {B} + slot", "        ")
        L.append("      }")
        # ---- prefetch the next iteration's edges; sender indices one more iteration ahead ----
        L.append("      { " + " ".join(f"const int t{k} = sender[min(e + {2 * nxt + k}, eend - 1)];"
                                       for k in range(len(sets))))
        for k, pf in enumerate(nsets):
            L += ld_xw(pf, f"e + {nxt + k}", f"s{k}", "      ")
        L.append(f"      const int es = (e - ebase) & {B - 1};")
        # ---- phase 2 ----
        L += compute(sets[0], "es", "      ")
        L.append("      ++e;")
        if PAIR:
            L += flush("      ")
            L.append("      if (e < eend) {")
            L += compute(sets[1], "es + 1", "        ")
            L.append("        ++e;")
            L.append("      }")
        L.append("      " + " ".join(f"{cs}{v} = {ns}{v};" for cs, ns in zip(sets, nsets) for v in xw_)
                 + " " + " ".join(f"s{k} = t{k};" for k in range(len(sets))) + " }")
        L.append("    }")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    return L


def _tp_path_cost(p: cg.TPPath) -> int:
    """VALU instructions per lane of one path in the per-lane CG form (_emit_acc), plus its
    operand reads: the balance weight of the cooperative forward's path partition."""
    nz = _path_cg(p)
    pairs = len({(i, j) for (i, j, k), _ in nz})
    iks = len({(i, k) for (i, j, k), _ in nz})
    d1, d2, d3 = 2 * p.l1 + 1, 2 * p.l2 + 1, 2 * p.l3 + 1
    return min(d3 + 1, d1, d2) + (pairs + len(nz) if pairs <= iks else len(nz) + iks) + 2


def coop_groups(paths: List[cg.TPPath], ng: int, max_acc: int) -> List[List[cg.TPPath]]:
    """Partition the paths into ``ng`` groups of balanced VALU cost (longest-processing-time
    greedy) with at most ``max_acc`` accumulators per lane each; within a group the paths are
    in (l1, l2, l3) order.  All groups of the cooperative forward meet at every batch barrier,
    so the slowest group sets the pace."""
    bins = [[0, 0, []] for _ in range(ng)]
    for p in sorted(paths, key=lambda p: (-_tp_path_cost(p), p.slot)):
        cand = [b for b in bins if b[1] + 2 * p.l3 + 1 <= max_acc]
        if not cand:
            raise ValueError(f"cannot place path {p} under {max_acc} accumulators in {ng} groups")
        b = min(cand, key=lambda b: (b[0], b[1]))
        b[0] += _tp_path_cost(p)
        b[1] += 2 * p.l3 + 1
        b[2].append(p)
    return [sorted(b[2], key=lambda p: (p.l1, p.l2, p.l3)) for b in bins if b[2]]


def tp_coop_shape(paths: List[cg.TPPath]) -> int:
    """Waves (= path groups) per block of the cooperative forward."""
    n = len(paths)
    return 8 if n >= 32 else 4 if n >= 12 else 2 if n >= 4 else 1


def emit_tp_fwd_coop(name, sfx, WT, ld_w, paths, din, nshp, wn, dmid, node_off, bf) -> Tuple[List[str], dict]:
    """Cooperative forward: one block = NG waves = NG balanced path groups, over two receiver
    tiles (lanes 0-31 of every wave on tile A, lanes 32-63 on tile B: the two halves of a wave
    run the same group's code on different receivers).

    The tiles' edges are staged in batches of TP_CO_BE edges per tile: for each edge the whole
    x[sender] row, the whole TP-weight row and the SH row are copied once into LDS by all the
    block's threads (float4 loads, issued a batch ahead into registers and written after the
    batch barrier), and every group wave reads its operands from there.  Against one block per
    path group (tp_fwd_m / the per-group kernel) each edge's rows cross L2 once instead of once
    per group, the weight rows stream contiguously, and the receivers' output rows are written
    by all groups at the same time (whole-row write locality).  Sender indices of a batch are
    staged in LDS one batch earlier still, so staging has no dependent global-load chain."""
    NG = tp_coop_shape(paths)
    groups = coop_groups(paths, NG, TP_CO_MAXACC)
    NG = len(groups)
    NT = 64 * NG
    BE = TP_CO_BE
    R = TP_CO_R
    es = 2 if bf else 4
    X4, W4, Y4 = din // 4, wn * es // 16, nshp // 4
    assert din % 4 == 0 and (wn * es) % 16 == 0 and nshp % 4 == 0
    ROW4 = X4 + W4 + Y4
    if ROW4 % 2 == 0:
        ROW4 += 1                         # odd row stride: the two tiles' rows start in other banks
    SLOTS = 2 * BE * ROW4
    # staging work: per kind (x rows, weight rows, SH rows) a compile-time run of float4 slots,
    # so every load's source kind is static (no per-slot branches or pointer selects)
    kinds = [("x", X4, 0), ("w", W4, X4), ("y", Y4, X4 + W4)]
    plan = []                                  # (kind, i): slot j = tid + NT * i of that kind
    for kd, n4, off in kinds:
        tot = 2 * BE * n4
        for i in range((tot + NT - 1) // NT):
            plan.append((kd, n4, off, i, tot))
    NS = len(plan)
    L: List[str] = []
    wpe = f" __attribute__((amdgpu_waves_per_eu({TP_CO_WPE})))" if TP_CO_WPE else ""
    L.append(f"__global__ __launch_bounds__({NT}){wpe} void tp_fwd_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ rowptr, int n_nodes,")
    L.append("    float inv_norm, float* __restrict__ agg) {")
    L.append(f"  __shared__ float4 st[{SLOTS}];")
    L.append(f"  __shared__ int sidx[{2 * BE}];")
    L.append("  const int tid = threadIdx.x, lane = tid & 63, u = lane & 31, h = lane >> 5;")
    # XCD-aware: the blocks of XCD k (blockIdx % 8 == k) take one contiguous range of tile pairs
    L.append(f"  const int nb = (n_nodes + {2 * R - 1}) / {2 * R}, nb8 = (nb + 7) >> 3;")
    L.append("  const int b = (blockIdx.x & 7) * nb8 + (blockIdx.x >> 3);")
    L.append("  if (b >= nb) return;")
    L.append(f"  const int rA = min(2 * b * {R}, n_nodes), rB = min(rA + {R}, n_nodes), rC = min(rB + {R}, n_nodes);")
    L.append("  const int eA = rowptr[rA], eB = rowptr[rB], eC = rowptr[rC];")
    L.append("  const int r0 = h ? rB : rA, r1 = h ? rC : rB, e0 = h ? eB : eA, e1 = h ? eC : eB;")
    L.append(f"  const int nbatch = (max(eB - eA, eC - eB) + {BE - 1}) / {BE};")
    L.append("  float4 " + ", ".join(f"sr{i}" for i in range(NS)) + ";")
    L.append("  int snext = 0;")

    def issue(bexpr, ind):
        """loads of batch ``bexpr`` (its sender indices already in sidx) into sr; sender indices
        of batch bexpr + 1 into snext"""
        # tid made opaque here: the per-slot index math is recomputed per batch (a few integer
        # ops) instead of being hoisted out of the batch loop into registers
        out = [f"{ind}{{ const int bb = {bexpr}; int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));"]
        out.append(f"{ind}  if (tid < {2 * BE}) {{ const int hh = tid / {BE}, k = tid - hh * {BE};")
        out.append(f"{ind}    const int e = (hh ? eB : eA) + (bb + 1) * {BE} + k, ee = hh ? eC : eB;")
        out.append(f"{ind}    snext = sender[min(e, max(ee - 1, 0))]; }}")
        for si, (kd, n4, off, i, tot) in enumerate(plan):
            out.append(f"{ind}  {{ const int j = min(tid + {NT * i}, {tot - 1});")
            out.append(f"{ind}    const int hk = j / {n4}, f = j - hk * {n4}, hh = hk / {BE}, k = hk - hh * {BE};")
            if kd == "x":
                out.append(f"{ind}    sr{si} = reinterpret_cast<const float4*>(x + (size_t)sidx[hk] * {din})[f]; }}")
            else:
                out.append(f"{ind}    const int e = min((hh ? eB : eA) + bb * {BE} + k, max((hh ? eC : eB) - 1, 0));")
                if kd == "w":
                    out.append(f"{ind}    sr{si} = reinterpret_cast<const float4*>(w + (size_t)e * {wn})[f]; }}")
                else:
                    out.append(f"{ind}    sr{si} = reinterpret_cast<const float4*>(sh + (size_t)e * {nshp})[f]; }}")
        out.append(f"{ind}}}")
        return out

    def commit(ind):
        out = [f"{ind}{{ int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));"]
        for si, (kd, n4, off, i, tot) in enumerate(plan):
            guard = f"tid + {NT * i} < {tot}" if NT * (i + 1) > tot else "true"
            out.append(f"{ind}{{ const int j = tid + {NT * i}; if ({guard}) {{ const int hk = j / {n4}; "
                       f"st[hk * {ROW4} + {off} + (j - hk * {n4})] = sr{si}; }} }}")
        out.append(f"{ind}if (tid < {2 * BE}) sidx[tid] = snext; }}")
        return out

    # prologue: sender indices of batch 0, then batch 0's rows (and batch 1's indices)
    L.append(f"  if (tid < {2 * BE}) {{ const int hh = tid / {BE}, k = tid - hh * {BE};")
    L.append(f"    const int e = (hh ? eB : eA) + k, ee = hh ? eC : eB;")
    L.append(f"    sidx[tid] = sender[min(e, max(ee - 1, 0))]; }}")
    L.append("  __syncthreads();")
    L += issue("0", "  ")
    L.append("  __syncthreads();")
    L += commit("  ")
    L.append("  __syncthreads();")
    L.append(f"  switch (tid >> 6) {{")
    only = os.environ.get("EELG_TP_CO_ONLY")           # register-budget probe: one group only
    for gi, grp in enumerate(groups):
        if only is not None and gi != int(only):
            continue
        need_l1 = sorted({p.l1 for p in grp})
        need_l2 = sorted({p.l2 for p in grp})
        accs = [f"a{p.slot}_{k}" for p in grp for k in range(2 * p.l3 + 1)]
        L.append(f"  case {gi}: {{ // {len(grp)} paths, {len(accs)} accumulators, cost {sum(_tp_path_cost(p) for p in grp)}")
        L.append("    float " + ", ".join(f"{a} = 0.0f" for a in accs) + ";")
        L.append("    int e = e0, node = r0;")
        L.append("    int nend = r0 < r1 ? rowptr[r0 + 1] : e1, nend2 = rowptr[min(r0 + 2, r1)];")

        def flush(ind):
            out = [f"{ind}while (node < r1 && nend == e) {{",
                   f"{ind}  float* __restrict__ o = agg + (size_t)node * {dmid};"]
            for p in grp:
                d3 = 2 * p.l3 + 1
                out.extend(f"{ind}  " + ln for ln in vec_store([f"a{p.slot}_{k}" for k in range(d3)], "o",
                                                              f"{p.out_off} + u * {d3}"))
            out.append(f"{ind}  " + " ".join(f"{a} = 0.0f;" for a in accs))
            out.append(f"{ind}  ++node; nend = nend2; nend2 = rowptr[min(node + 2, r1)];")
            out.append(f"{ind}}}")
            return out
        L.append("    for (int bi = 0; bi < nbatch; ++bi) {")
        L += issue("bi + 1", "      ")
        L.append(f"      const int kend = min({BE}, e1 - e);")
        L.append("      for (int k = 0; k < kend; ++k) {")
        L += flush("        ")
        L.append(f"        const float4* __restrict__ rw = st + (h * {BE} + k) * {ROW4};")
        L.append("        const float* __restrict__ xs = reinterpret_cast<const float*>(rw);")
        L.append(f"        const {WT}* __restrict__ we = reinterpret_cast<const {WT}*>(rw + {X4}) + u;")
        L.append(f"        const float* __restrict__ ye = reinterpret_cast<const float*>(rw + {X4 + W4});")
        # operands are read from LDS per path (short live ranges: registers), the pins after
        # each path keep the reads there
        xn = lambda p, i: f"px{i}"  # noqa: E731
        yn = lambda p, j: f"py{j}"  # noqa: E731
        for p in grp:
            d1, d2, d3 = 2 * p.l1 + 1, 2 * p.l2 + 1, 2 * p.l3 + 1
            L.append(f"        {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
            L.append("          " + " ".join(f"const float px{i} = xs[{node_off[p.l1]} + u * {d1} + {i}];"
                                             for i in range(d1)))
            L.append("          float " + ", ".join(f"py{j}" for j in range(d2)) + ";")
            L += ["          " + ln for ln in vec_load([f"py{j}" for j in range(d2)], "ye", str(p.l2 * p.l2))]
            L.append(f"          const float wp = {ld_w(f'we[{p.slot * MUL}]')} * ({flit(p.coef)} * inv_norm);")
            fold = min((d3 + 1, "none"), (d1, "x"), (d2, "y"))
            if fold[1] == "none":
                _emit_t(p, xn, yn, "t", L, "          ")
                for k in range(d3):
                    L.append(f"          a{p.slot}_{k} = fmaf(wp, t{k}, a{p.slot}_{k});")
            else:
                if fold[1] == "x":
                    for i in range(d1):
                        L.append(f"          const float xw{i} = {xn(p, i)} * wp;")
                    xf, yf = (lambda p, i: f"xw{i}"), yn
                else:
                    for j in range(d2):
                        L.append(f"          const float yw{j} = {yn(p, j)} * wp;")
                    xf, yf = xn, (lambda p, j: f"yw{j}")
                _emit_acc(p, xf, yf, lambda k, p=p: f"a{p.slot}_{k}", L, "          ")
            L.append("        }")
            L.append("        " + pin(accs, memory=True))
        L.append("        ++e;")
        L.append("      }")
        L.append("      __syncthreads();")
        L += commit("      ")
        L.append("      __syncthreads();")
        L.append("    }")
        L += flush("    ")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    return L, {"fwd_threads": NT, "fwd_tile": 2 * R, "ngroups": NG}


def emit_tp(name: str, node: Irreps, sh: Irreps, target: Irreps, wt: str = "f32") -> Tuple[str, dict]:
    """``wt`` = "f32" | "bf16": storage type of the edge-sized tensors (TP weights w and
    grad_w, per-edge grad gxe); arithmetic is fp32 either way (BASELINE config 5)."""
    bf = wt == "bf16"
    sfx = "_bw" if bf else ""
    WT = "unsigned short" if bf else "float"
    ld_w = (lambda e: f"eelg_bf2f({e})") if bf else (lambda e: e)   # noqa: E731
    st_w = (lambda v: f"eelg_f2bf({v})") if bf else (lambda v: v)   # noqa: E731
    paths = cg.tp_paths(node, sh, target)
    din, nsh = node.dim, sh.dim
    nshp = (nsh + 3) // 4 * 4              # padded SH row stride (float4 loads)
    irreps_mid = cg.tp_out_irreps_with_instructions(node, sh, target)[0]
    dmid = irreps_mid.dim
    wn = sum(p.mul for p in paths)
    for p in paths:
        assert p.mul == MUL
    pk2 = TP_PK2 and [ir.l for _, ir in node] != [0]
    groups = _group_paths(sorted(paths, key=lambda p: (p.l1, p.l2, p.l3)),
                          TP_PK2_MAXACC if pk2 else TP_MAXACC)
    node_ls = [ir.l for _, ir in node]
    node_off = {ir.l: o for (m, ir), o in zip(node, node.offsets())}
    L: List[str] = []
    L.append(f"// ===== tensor product config {name}: {node} (x) {sh} -> {irreps_mid} =====")
    L.append(f"// {len(paths)} 'uvu' paths, weight_numel {wn}, {len(groups)} path groups")
    xname = lambda p, i: f"x{p.l1}_{i}"  # noqa: E731
    yname = lambda p, j: f"y{p.l2 * p.l2 + j}"  # noqa: E731

    # ---------------- forward ----------------
    # One half-wave (32 lanes = 32 channels) owns TP_NPH consecutive receivers.  Edges are
    # receiver-sorted, so their in-edges form ONE contiguous range that the half-wave
    # streams through with a software pipeline (sender index two edges ahead, the gathered
    # x / SH / weight row one edge ahead); at each receiver boundary the register
    # accumulators are stored and reset.  The latency chain rowptr -> sender -> x is paid
    # once per TP_NPH receivers instead of once per receiver.  Blocks are numbered so that
    # the ngroups path-group blocks of one node tile share blockIdx.x % 8, i.e. one XCD,
    # and read the tile's x rows / SH rows / indices through one L2.
    ng = len(groups)
    coop = None
    if TP_PK2 and node_ls != [0]:
        L += emit_tp_fwd_pk2(name, sfx, WT, bf, groups, din, nshp, wn, dmid, node_off)
        fwd_done = True
    elif TP_COOP:
        code, coop = emit_tp_fwd_coop(name, sfx, WT, ld_w, paths, din, nshp, wn, dmid, node_off, bf)
        L += code
        fwd_done = True
    elif TP_FWD_M:
        L += emit_tp_fwd_m(name, sfx, WT, ld_w, groups, din, nshp, nsh, wn, dmid, node_off)
        fwd_done = True
    else:
        fwd_done = False
    wpe = f" __attribute__((amdgpu_waves_per_eu({TP_WPE})))" if TP_WPE else ""
    L.append(f"__global__ __launch_bounds__(256){wpe} void tp_fwd_{name}{sfx}{'_unused' if fwd_done else ''}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ rowptr, int n_nodes,")
    L.append("    float inv_norm, float* __restrict__ agg) {")
    L.append("  const int lane = threadIdx.x & 63;")
    L.append(f"  const int u = lane & {MUL - 1};")
    L.append(f"  const int q = blockIdx.x >> 3, grp = q % {ng};")
    if TP_XCD_CONTIG:
        # XCD k (blockIdx % 8) takes one contiguous range of node tiles, walked in order: the
        # x rows of a lattice are gathered by one XCD (its L2) rather than by all eight
        L.append(f"  const int ntl = (n_nodes + {8 * TP_NPH - 1}) / {8 * TP_NPH}, tpx = (ntl + 7) >> 3;")
        L.append(f"  const int tile = (blockIdx.x & 7) * tpx + q / {ng};")
    else:
        L.append(f"  const int tile = (q / {ng}) * 8 + (blockIdx.x & 7);")
    L.append(f"  const int n0 = ((tile * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5)) * {TP_NPH};")
    L.append("  if (n0 >= n_nodes) return;")
    L.append(f"  const int n1 = min(n0 + {TP_NPH}, n_nodes);")
    L.append("  switch (grp) {")
    for gi, grp in enumerate(groups):
        L.append(f"  case {gi}: {{")
        need_l1 = sorted({p.l1 for p in grp})
        need_l2 = sorted({p.l2 for p in grp})
        accs = [f"a{p.slot}_{k}" for p in grp for k in range(2 * p.l3 + 1)]
        L.append("    float " + ", ".join(f"{a} = 0.0f" for a in accs) + ";")
        cur = ([f"x{l}_{i}" for l in need_l1 for i in range(2 * l + 1)]
               + [f"y{l * l + j}" for l in need_l2 for j in range(2 * l + 1)]
               + [f"w{p.slot}" for p in grp])

        def load(pref, ev, sv, guard):
            # addresses stay in bounds when the edge does not exist (index 0); the loaded
            # values of a missing edge are never used
            out = [f"    {{ const bool ok = {guard};",
                   f"      const float* __restrict__ xs = x + (size_t){sv} * {din};",
                   f"      const float* __restrict__ ye = sh + (size_t)(ok ? {ev} : 0) * {nshp};",
                   f"      const {WT}* __restrict__ we = w + (size_t)(ok ? {ev} : 0) * {wn} + u;"]
            for l in need_l1:
                d = 2 * l + 1
                out += ["      " + ln for ln in vec_load([f"{pref}x{l}_{i}" for i in range(d)], "xs",
                                                          f"{node_off[l]} + u * {d}")]
            out += ["      " + ln for ln in sh_load(need_l2, pref, "ye")]
            for p in grp:
                out.append(f"      {pref}w{p.slot} = {ld_w(f'we[{p.slot * MUL}]')};")
            out.append("    }")
            return out
        L.append("    int e = rowptr[n0];")
        L.append("    const int eend = rowptr[n1];")
        L.append("    int node = n0, nend = rowptr[n0 + 1], nend2 = rowptr[min(n0 + 2, n1)];")
        L.append("    int s1 = e + 1 < eend ? sender[e + 1] : 0;")
        L.append("    float " + ", ".join(cur) + ";")
        L += load("", "e", "(e < eend ? sender[e] : 0)", "e < eend")
        gpin = pin(accs + cur)
        def step(cp, np_):
            """one pipelined edge step: flush finished receivers, issue edge e+1's loads
            into the ``np_`` register set, compute edge e from the ``cp`` set"""
            out = []
            # flush every receiver whose range ends here (also covers receivers with no in-edges)
            out.append("      while (node < n1 && nend == e) {")
            out.append(f"        float* __restrict__ o = agg + (size_t)node * {dmid};")
            for p in grp:
                d3 = 2 * p.l3 + 1
                out.extend("        " + ln for ln in vec_store([f"a{p.slot}_{k}" for k in range(d3)], "o",
                                                             f"{p.out_off} + u * {d3}"))
            out.append("        " + " ".join(f"{a} = 0.0f;" for a in accs))
            out.append("        ++node; nend = nend2; nend2 = rowptr[min(node + 2, n1)];")
            out.append("      }")
            out.append("      if (e >= eend) break;")
            out.append("      { const int s2 = e + 2 < eend ? sender[e + 2] : 0;")
            out.extend("  " + ln for ln in load(np_, "e + 1", "s1", "e + 1 < eend"))
            cpin = pin(accs + [cp + v for v in cur] + ([] if TP_NOPIN_NEXT else [np_ + v for v in cur]))
            # TP_PIN_NEXT_LAST: the in-flight next-edge registers are pinned only after the
            # last path, so no earlier path boundary waits for the prefetch to land
            cpin_mid = pin(accs + [cp + v for v in cur]) if TP_PIN_NEXT_LAST else cpin
            xn = lambda p, i: f"{cp}x{p.l1}_{i}"  # noqa: E731
            yn = lambda p, j: f"{cp}y{p.l2 * p.l2 + j}"  # noqa: E731
            if TP_NOCOMPUTE:
                # diagnostic (memory-pattern floor): every loaded value feeds one sum that is
                # added to every accumulator; the loads, stores and loop are tp_fwd's own
                out.append("      { const float z_ = " + " + ".join(cp + v for v in cur) + ";")
                out.append("        " + " ".join(f"{a} += z_;" for a in accs) + " }")
                out.append("      " + cpin)
            for p in ([] if TP_NOCOMPUTE else grp):
                d1, d2, d3 = 2 * p.l1 + 1, 2 * p.l2 + 1, 2 * p.l3 + 1
                out.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
                out.append(f"        const float wp = {cp}w{p.slot} * ({flit(p.coef)} * inv_norm);")
                fold = min((d3 + 1, "none"), (d1, "x"), (d2, "y")) if TP_FOLDW else (0, "none")
                if fold[1] == "none":
                    _emit_t(p, xn, yn, "t", out, "        ")
                    for k in range(d3):
                        out.append(f"        a{p.slot}_{k} = fmaf(wp, t{k}, a{p.slot}_{k});")
                else:
                    # fold the path weight into the shorter of x / y (d1 or d2 products instead
                    # of d3 + 1) and accumulate the CG terms straight into the accumulators
                    if fold[1] == "x":
                        for i in range(d1):
                            out.append(f"        const float xw{i} = {xn(p, i)} * wp;")
                        xf, yf = (lambda p, i: f"xw{i}"), yn
                    else:
                        for j in range(d2):
                            out.append(f"        const float yw{j} = {yn(p, j)} * wp;")
                        xf, yf = xn, (lambda p, j: f"yw{j}")
                    _emit_acc(p, xf, yf, lambda k, p=p: f"a{p.slot}_{k}", out, "        ")
                out.append("      }")
                out.append("      " + (cpin if p is grp[-1] else cpin_mid))
            out.append("      s1 = s2; ++e; }")
            return out
        if TP_UNROLL2:
            # two register sets, alternating roles: no end-of-iteration copies
            L.append("    float " + ", ".join("n" + v for v in cur) + ";")
            L.append("    for (;;) {")
            L += step("", "n")
            L += step("n", "")
            L.append("    }")
        else:
            L.append("    for (;;) {")
            L.append("      float " + ", ".join("n" + v for v in cur) + ";")
            L += step("", "n")
            L.append("      " + " ".join(f"{v} = n{v};" for v in cur))
            L.append("    }")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")

    # ---------------- backward (per edge) ----------------
    # grouped by input block l1: each group owns a disjoint slice of gxe, so no
    # cross-group reduction is needed; grad_w of every path is written once.
    bgroups = [[p for p in paths if p.l1 == l] for l in node_ls]
    bgroups = [g for g in bgroups if g]
    L.append(f"__global__ __launch_bounds__(256) void tp_bwd_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ receiver, int n_edges,")
    L.append("    const float* __restrict__ gagg, float inv_norm,")
    L.append(f"    {WT}* __restrict__ gw, {WT}* __restrict__ gxe, const int* __restrict__ spos) {{")
    L.append("  const int lane = threadIdx.x & 63;")
    L.append(f"  const int u = lane & {MUL - 1};")
    # spos (optional): gxe row of edge e is spos[e], its position in sender order, so the sender
    # sum reads gxe contiguously instead of gathering rows through sperm
    # a half-wave streams TP_BWD_EPH consecutive edges: while the last path of edge e
    # computes, edge e+1's x / SH rows and first path's grad_agg slice and weight are in
    # flight (its sender / receiver indices were loaded when edge e started)
    EPH = TP_BWD_EPH
    L.append(f"  const int e0 = ((blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5)) * {EPH};")
    L.append("  if (e0 >= n_edges) return;")
    L.append(f"  const int e1 = min(e0 + {EPH}, n_edges);")
    L.append("  switch (blockIdx.y) {")
    for gi, grp in enumerate(bgroups):
        l = grp[0].l1
        d = 2 * l + 1
        l2s = sorted({p.l2 for p in grp})
        xs_ = [f"x{l}_{i}" for i in range(d)]
        ys_ = [f"y{l2 * l2 + j}" for l2 in l2s for j in range(2 * l2 + 1)]
        p0 = grp[0]
        g0_ = [f"g{p0.slot}_{k}" for k in range(2 * p0.l3 + 1)] + [f"w{p0.slot}"]
        L.append(f"  case {gi}: {{ // input block l1 = {l}")

        def edge_loads(pref, sv, rv, ev):
            """x / SH rows of an edge and its first path's grad_agg slice + weight"""
            out = [f"    {{ const float* __restrict__ xs = x + (size_t){sv} * {din};",
                   f"      const float* __restrict__ ye = sh + (size_t){ev} * {nshp};",
                   f"      const float* __restrict__ ge = gagg + (size_t){rv} * {dmid};",
                   f"      const {WT}* __restrict__ we = w + (size_t){ev} * {wn} + u;"]
            out += ["      " + ln for ln in vec_load([pref + v for v in xs_], "xs", f"{node_off[l]} + u * {d}")]
            out += ["      " + ln for ln in sh_load(l2s, pref, "ye")]
            d3 = 2 * p0.l3 + 1
            out += ["      " + ln for ln in vec_load([f"{pref}g{p0.slot}_{k}" for k in range(d3)], "ge",
                                                      f"{p0.out_off} + u * {d3}")]
            out.append(f"      {pref}w{p0.slot} = {ld_w(f'we[{p0.slot * MUL}]')};")
            out.append("    }")
            return out
        L.append("    float " + ", ".join(xs_ + ys_ + g0_) + ";")
        L.append("    int rcur = receiver[e0];")
        L += edge_loads("", "sender[e0]", "rcur", "e0")
        L.append("    for (int e = e0; e < e1; ++e) {")
        if EPH > 1:
            L.append("      const bool more = e + 1 < e1;")
            L.append("      const int sn = more ? sender[e + 1] : 0, rn = more ? receiver[e + 1] : 0;")
            L.append("      const int en = more ? e + 1 : e;")
        L.append("      const float* __restrict__ ge = gagg + (size_t)rcur * " + str(dmid) + ";")
        L.append(f"      const {WT}* __restrict__ we = w + (size_t)e * {wn} + u;")
        L.append(f"      {WT}* __restrict__ gwe = gw + (size_t)e * {wn} + u;")
        L.append(f"      {WT}* __restrict__ gxo = gxe + (size_t)(spos ? spos[e] : e) * {din};")
        for i in range(d):
            L.append(f"      float gx{l}_{i} = 0.0f;")
        if EPH > 1:
            L.append("      float " + ", ".join("n" + v for v in xs_ + ys_ + g0_) + ";")
        base_pin = xs_ + [f"gx{l}_{i}" for i in range(d)] + ys_

        def pref(p):
            """issue the loads one path needs (its grad_agg slot row and weight)"""
            d3 = 2 * p.l3 + 1
            out = ["      float " + ", ".join(f"g{p.slot}_{k}" for k in range(d3)) + ";"]
            out += ["      " + ln for ln in vec_load([f"g{p.slot}_{k}" for k in range(d3)], "ge",
                                                    f"{p.out_off} + u * {d3}")]
            out.append(f"      float w{p.slot} = {ld_w(f'we[{p.slot * MUL}]')};")
            return out, [f"g{p.slot}_{k}" for k in range(d3)] + [f"w{p.slot}"]
        for pi, p in enumerate(grp):
            d3 = 2 * p.l3 + 1
            d1 = 2 * p.l1 + 1
            if pi + 1 < len(grp):            # next path's loads in flight during this one
                code, nxt_regs = pref(grp[pi + 1])
                L += code
            elif EPH > 1:                    # next edge's loads in flight during the last path
                L += ["  " + ln for ln in edge_loads("n", "sn", "rn", "en")]
                nxt_regs = ["n" + v for v in xs_ + ys_ + g0_]
            else:
                nxt_regs = []
            L.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
            L.append(f"        const float cp = {flit(p.coef)} * inv_norm;")
            nz = _path_cg(p)
            byik: Dict[Tuple[int, int], List[str]] = {}
            for (i, j, k), c in nz:
                byik.setdefault((i, k), []).append(f"{flit(c)} * y{p.l2 * p.l2 + j}")
            for (i, k), ts in byik.items():
                L.append(f"        const float m{i}_{k} = {' + '.join(ts)};")
            gterms = []
            for k in range(d3):
                ts = [f"x{p.l1}_{i} * m{i}_{k}" for i in range(d1) if (i, k) in byik]
                if ts:
                    gterms.append(f"g{p.slot}_{k} * ({' + '.join(ts)})")
            gexpr = " + ".join(gterms) if gterms else "0.0f"
            L.append(f"        gwe[{p.slot * MUL}] = {st_w(f'cp * ({gexpr})')};")
            L.append(f"        const float hw = cp * w{p.slot};")
            for i in range(d1):
                ts = [f"m{i}_{k} * g{p.slot}_{k}" for k in range(d3) if (i, k) in byik]
                if ts:
                    L.append(f"        gx{p.l1}_{i} = fmaf(hw, {' + '.join(ts)}, gx{p.l1}_{i});")
            L.append("      }")
            L.append("      " + pin(base_pin + nxt_regs))
        if bf:
            L += [f"      gxo[{node_off[l]} + u * {d} + {i}] = eelg_f2bf(gx{l}_{i});" for i in range(d)]
        else:
            L += ["      " + ln for ln in vec_store([f"gx{l}_{i}" for i in range(d)], "gxo", f"{node_off[l]} + u * {d}")]
        if EPH > 1:
            L.append("      " + " ".join(f"{v} = n{v};" for v in xs_ + ys_ + g0_) + " rcur = rn;")
        L.append("    }")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")

    # ---------------- backward in sender order ----------------
    # One half-wave owns one SENDER node and walks its out-edges through the sender CSR
    # (srowptr / sperm): x[sender] is loaded once, grad_x is summed in registers and stored
    # once per node, so the per-edge gxe [E, din] round trip and the segment sum that read
    # it back disappear.  grad_w is written at each edge's own row as before.  Summation
    # order over a sender's edges is the sperm order, the same as segment_sum_csr's.
    L.append(f"__global__ __launch_bounds__(256) void tp_bws_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sperm, const int* __restrict__ srowptr,")
    L.append("    const int* __restrict__ receiver, int n_nodes,")
    L.append("    const float* __restrict__ gagg, float inv_norm,")
    L.append(f"    {WT}* __restrict__ gw, float* __restrict__ gx) {{")
    L.append("  const int lane = threadIdx.x & 63;")
    L.append(f"  const int u = lane & {MUL - 1};")
    L.append("  const int n = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);")
    L.append("  if (n >= n_nodes) return;")
    L.append("  const int p0 = srowptr[n], p1 = srowptr[n + 1];")
    L.append("  switch (blockIdx.y) {")
    for gi, grp in enumerate(bgroups):
        l = grp[0].l1
        d = 2 * l + 1
        l2s = sorted({p.l2 for p in grp})
        xs_ = [f"x{l}_{i}" for i in range(d)]
        ys_ = [f"y{l2 * l2 + j}" for l2 in l2s for j in range(2 * l2 + 1)]
        gxs = [f"gx{l}_{i}" for i in range(d)]
        L.append(f"  case {gi}: {{ // input block l1 = {l}")
        L.append("    float " + ", ".join(xs_) + ";")
        L.append(f"    {{ const float* __restrict__ xs = x + (size_t)n * {din};")
        L += ["      " + ln for ln in vec_load(xs_, "xs", f"{node_off[l]} + u * {d}")]
        L.append("    }")
        L.append("    float " + ", ".join(f"{v} = 0.0f" for v in gxs) + ";")
        L.append("    int en = p0 < p1 ? sperm[p0] : 0;")
        L.append("    for (int p = p0; p < p1; ++p) {")
        L.append("      const int e = en;")
        L.append("      en = p + 1 < p1 ? sperm[p + 1] : 0;")
        L.append("      const int r = receiver[e];")
        L.append(f"      const float* __restrict__ ye = sh + (size_t)e * {nshp};")
        L.append(f"      const float* __restrict__ ge = gagg + (size_t)r * {dmid};")
        L.append(f"      const {WT}* __restrict__ we = w + (size_t)e * {wn} + u;")
        L.append(f"      {WT}* __restrict__ gwe = gw + (size_t)e * {wn} + u;")
        L.append("      float " + ", ".join(ys_) + ";")
        L += ["      " + ln for ln in sh_load(l2s, "", "ye")]

        def pload(p):
            d3 = 2 * p.l3 + 1
            out = ["      float " + ", ".join(f"g{p.slot}_{k}" for k in range(d3)) + ";"]
            out += ["      " + ln for ln in vec_load([f"g{p.slot}_{k}" for k in range(d3)], "ge",
                                                    f"{p.out_off} + u * {d3}")]
            out.append(f"      float w{p.slot} = {ld_w(f'we[{p.slot * MUL}]')};")
            return out, [f"g{p.slot}_{k}" for k in range(d3)] + [f"w{p.slot}"]
        code, _ = pload(grp[0])
        L += code
        for pi, p in enumerate(grp):
            d3 = 2 * p.l3 + 1
            d1 = 2 * p.l1 + 1
            nxt_regs = []
            if pi + 1 < len(grp):            # next path's loads in flight during this one
                code, nxt_regs = pload(grp[pi + 1])
                L += code
            L.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
            L.append(f"        const float cp = {flit(p.coef)} * inv_norm;")
            byik: Dict[Tuple[int, int], List[str]] = {}
            for (i, j, k), c in _path_cg(p):
                byik.setdefault((i, k), []).append(f"{flit(c)} * y{p.l2 * p.l2 + j}")
            for (i, k), ts in byik.items():
                L.append(f"        const float m{i}_{k} = {' + '.join(ts)};")
            gterms = []
            for k in range(d3):
                ts = [f"x{p.l1}_{i} * m{i}_{k}" for i in range(d1) if (i, k) in byik]
                if ts:
                    gterms.append(f"g{p.slot}_{k} * ({' + '.join(ts)})")
            gexpr = " + ".join(gterms) if gterms else "0.0f"
            L.append(f"        gwe[{p.slot * MUL}] = {st_w(f'cp * ({gexpr})')};")
            L.append(f"        const float hw = cp * w{p.slot};")
            for i in range(d1):
                ts = [f"m{i}_{k} * g{p.slot}_{k}" for k in range(d3) if (i, k) in byik]
                if ts:
                    L.append(f"        gx{p.l1}_{i} = fmaf(hw, {' + '.join(ts)}, gx{p.l1}_{i});")
            L.append("      }")
            L.append("      " + pin(xs_ + gxs + ys_ + nxt_regs))
        L.append("    }")
        L.append(f"    float* __restrict__ gxo = gx + (size_t)n * {din};")
        L += ["    " + ln for ln in vec_store(gxs, "gxo", f"{node_off[l]} + u * {d}")]
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    info = dict(din=din, dmid=dmid, wn=wn, nsh=nsh, ngroups=len(groups), nbgroups=len(bgroups),
                npaths=len(paths), nph=2 * TP_NPH if pk2 else TP_NPH, beph=TP_BWD_EPH,
                sig=fnv1a64(tp_signature(node, sh, target)),
                fwd_threads=coop["fwd_threads"] if coop else 256, fwd_tile=coop["fwd_tile"] if coop else 0)
    if coop:
        info["ngroups"] = coop["ngroups"]
    return "\n".join(L), info


# ---------------------------------------------------------------------------
# symmetric contraction
# ---------------------------------------------------------------------------
def pin(vs: List[str], memory: bool = False, sgprs: Sequence[str] = ()) -> str:
    if SC_PK == 3 and PIN_FIELDS:
        vs = [f for v in vs for f in ((v,) if v.startswith("acc[") or v.startswith("red[") else
                                      (f"{v}.x", f"{v}.y"))]
    return _pin(vs, memory, sgprs)


PIN_FIELDS = False      # set while emitting the SC_PK=3 fwd / grad-x bodies


def _pin(vs: List[str], memory: bool = False, sgprs: Sequence[str] = ()) -> str:
    """Empty asm that 'modifies' every listed register: a hard boundary for the
    scheduler, so each term block computes in place (without it hipcc hoists
    thousands of monomials / scalar coefficient loads and spills).  ``sgprs`` are
    wave-uniform values forced to be resident (loaded) at this point."""
    out = []
    ops_all = [f'"+v"({v})' for v in vs] + [f'"+s"({v})' for v in sgprs]
    for k in range(0, len(ops_all), 10):
        ops = ", ".join(ops_all[k: k + 10])
        out.append(f'asm volatile("" : {ops}{" : : " + chr(34) + "memory" + chr(34) if memory else ""});')
    return " ".join(out)


def sc_blocks(plan, maxb: int = 32) -> List[Dict]:
    """Split the polynomial terms into blocks of <= maxb terms (one (a, b) group may span
    several blocks; a c-subgroup is never split).  Each block's coefficients are
    prefetched into SGPRs while the previous block computes."""
    deg1, pairs = [], {}
    for t, (nu, (a, b, c), q) in enumerate(plan.terms):
        if nu == 1:
            deg1.append((t, a, q))
        else:
            g = pairs.setdefault((a, b), {"d2": [], "d3": {}})
            if nu == 2:
                g["d2"].append((t, q))
            else:
                g["d3"].setdefault(c, []).append((t, q))
    blocks = []
    if deg1:
        blocks.append({"kind": "deg1", "terms": [t for t, _, _ in deg1], "deg1": deg1})
    for (a, b), g in pairs.items():
        cur = {"kind": "pair", "a": a, "b": b, "first": True, "last": False,
               "d2": list(g["d2"]), "d3": [], "terms": [t for t, _ in g["d2"]]}
        for c, lst in g["d3"].items():
            if cur["terms"] and len(cur["terms"]) + len(lst) > maxb:
                blocks.append(cur)
                cur = {"kind": "pair", "a": a, "b": b, "first": False, "last": False,
                       "d2": [], "d3": [], "terms": []}
            cur["d3"].append((c, lst))
            cur["terms"] += [t for t, _ in lst]
        cur["last"] = True
        blocks.append(cur)
    return blocks


def emit_sc(name: str, coupling: str, ls: Tuple[int, ...], corr: int) -> Tuple[str, dict]:
    """Symmetric contraction kernels.

    Layout: x / out rows are e3nn mul-major ([l-block][channel][m]); a workgroup
    of 4 waves owns 4 consecutive channels ("channel quad") x 64 nodes and stages
    the quad's 4*D floats per node through LDS with contiguous global segments, so
    every byte of x / out crosses HBM once.  One wave = one channel (wave-uniform,
    coefficients come through scalar loads), one lane = one node.  The output irreps
    (``ls``, parity (-1)^l) may differ from the coupling irreps of the input (the
    reference's product block maps the interaction irreps onto the hidden irreps)."""
    global PIN_FIELDS
    PIN_FIELDS = SC_PK == 3
    try:
        return _emit_sc(name, coupling, ls, corr)
    finally:
        PIN_FIELDS = False


def _emit_sc(name: str, coupling: str, ls: Tuple[int, ...], corr: int) -> Tuple[str, dict]:
    plan = cg.symcon_plan(coupling, ls, corr)
    irs = [ir for _, ir in Irreps(coupling)]
    out_irs = [Ir(l, (-1) ** l) for l in ls]
    Q = 4                                   # channels per workgroup

    class Lay:
        """per-channel component list of one row layout (q channels per workgroup tile)"""
        def __init__(self, irreps, tag, q=4):
            Q = q
            self.comp, off, seg = [], 0, 0   # component a -> (l, m, row offset, seg start)
            self.segs = []
            for ir in irreps:
                for m in range(ir.dim):
                    self.comp.append((ir.l, m, off, seg))
                self.segs.append((seg, seg + Q * ir.dim, off, ir.dim))
                off += MUL * ir.dim
                seg += Q * ir.dim
            self.D = len(self.comp)
            self.QD = Q * self.D
            self.row = off
            self.goff = f"sc_goff_{name}_{tag}"

    lin, lout = Lay(irs, "in"), Lay(out_irs, "out")
    D, Dout = lin.D, lout.D
    TP = max(lin.QD, lout.QD) + 1           # padded LDS row shared by in / out tiles
    if TP % 2 == 0:
        TP += 1                             # odd -> conflict-free lane rows
    drow, orow = lin.row, lout.row
    nt = len(plan.terms)

    def lq(lay, a, cl):
        """LDS column of component a for channel-in-quad cl (may be a runtime expr)."""
        l, m, _, sg = lay.comp[a]
        return f"{sg} + ({cl}) * {2 * l + 1} + {m}"

    L: List[str] = []
    L.append(f"// ===== symmetric contraction config {name}: coupling {coupling} -> ls {ls}, correlation {corr} =====")
    L.append(f"// {nt} polynomial terms per channel; rows of {drow} -> {orow} floats")

    # global offset of quad-tile column q for channel quad cq (per layout)
    for lay in ((lin,) if lout.comp == lin.comp else (lin, lout)):
        L.append(f"__device__ __forceinline__ int {lay.goff}(int q, int cq) {{")
        for (a, b, o, d) in lay.segs[:-1]:
            L.append(f"  if (q < {b}) return {o} + cq * {Q * d} + (q - {a});")
        a, b, o, d = lay.segs[-1]
        L.append(f"  return {o} + cq * {Q * d} + (q - {a});")
        L.append("}")
    if lout.comp == lin.comp:
        lout.goff = lin.goff

    # SC_PK: 1 = one node per lane; 2 = two nodes per lane in packed fp32 (v_pk_*); 3 = two
    # nodes per lane in plain fp32 (a two-float struct: every coefficient scalar load and LDS
    # coefficient fetch feeds two independent FMAs, no packed-operand constraints)
    PKN = 2 if SC_PK in (2, 3) else 1
    # node tiles per workgroup (fwd / grad-x): waves w and w + 4 run the same channel on two
    # 64-node tiles, so the second wave's coefficient scalar loads hit the scalar cache line
    # the first one brought in
    NT = SC_NT if PKN == 1 else 1
    NB = 64 * PKN * NT                      # nodes per workgroup (fwd / grad-x)
    NTH = 256 * NT                          # threads per workgroup
    FT = {1: "float", 2: "eelg_f2", 3: "eelg_d2"}[SC_PK]
    ZERO = "0.0f" if PKN == 1 else f"{FT}{{0.0f, 0.0f}}"

    def fma_s(c, v, acc):
        """acc + c * v, c a wave-uniform scalar coefficient"""
        return f"fmaf({c}, {v}, {acc})" if PKN == 1 else f"eelg_fma2s({c}, {v}, {acc})"

    def fma_v(a, b, acc):
        return f"fmaf({a}, {b}, {acc})" if PKN == 1 else f"eelg_fma2({a}, {b}, {acc})"

    def ld_pair(dst, base0, base1, col):
        if PKN == 1:
            return f"{FT} {dst} = {base0}[{col}];"
        return f"{FT} {dst} = {FT}{{{base0}[{col}], {base1}[{col}]}};"

    def st_pair(val, base0, base1, col):
        if PKN == 1:
            return f"{base0}[{col}] = {val};"
        return f"{base0}[{col}] = {val}.x; {base1}[{col}] = {val}.y;"

    def stage_in(src, tile, lay, nb=64, nth=256):
        per = (nb * lay.QD + nth - 1) // nth
        out = ["  { int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));",
               "#pragma unroll 2",
               f"  for (int it = 0; it < {per}; ++it) {{",
               f"    const int idx = tid + {nth} * it;",
               f"    if (idx < {nb * lay.QD}) {{",
               f"      const int nl = idx / {lay.QD}, q = idx - nl * {lay.QD}, n = n0 + nl;",
               f"      {tile}[nl * {TP} + q] = (n < n_nodes) ? {src}[(size_t)n * {lay.row} + {lay.goff}(q, cq)] : 0.0f;",
               "    }", "  } }"]
        return out

    def stage_out(dst, tile, lay, nb=64, nth=256):
        per = (nb * lay.QD + nth - 1) // nth
        return ["  { int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));",
                "#pragma unroll 2",
                f"  for (int it = 0; it < {per}; ++it) {{",
                f"    const int idx = tid + {nth} * it;",
                f"    if (idx < {nb * lay.QD}) {{",
                f"      const int nl = idx / {lay.QD}, q = idx - nl * {lay.QD}, n = n0 + nl;",
                f"      if (n < n_nodes) {dst}[(size_t)n * {lay.row} + {lay.goff}(q, cq)] = {tile}[nl * {TP} + q];",
                "    }", "  } }"]

    def cm_store(dst, tile, lay, nb, ind="  ", nth=256):
        """dst[(c * D + a) * n_nodes + n] = component a of channel c of node n, from a staged
        tile of nb nodes x the quad's 4 channels (coalesced nb-float runs per (c, a))"""
        dd = lay.D
        sgs = ", ".join(str(lay.comp[a][3]) for a in range(dd))
        dls = ", ".join(str(2 * lay.comp[a][0] + 1) for a in range(dd))
        ms = ", ".join(str(lay.comp[a][1]) for a in range(dd))
        sh = nb.bit_length() - 1
        per = (Q * dd * nb + nth - 1) // nth
        out = [f"{{ const int kseg[{dd}] = {{{sgs}}}, kd[{dd}] = {{{dls}}}, km[{dd}] = {{{ms}}};",
               f"  for (int it = 0; it < {per}; ++it) {{",
               f"    const int idx = threadIdx.x + {nth} * it;",
               f"    if (idx < {Q * dd * nb}) {{",
               f"      const int row = idx >> {sh}, nl = idx & {nb - 1}, n = n0 + nl;",
               f"      const int cl = row / {dd}, a = row - cl * {dd};",
               f"      if (n < n_nodes) {dst}[(size_t)((cq * {Q} + cl) * {dd} + a) * n_nodes + n] = "
               f"{tile}[nl * {TP} + kseg[a] + cl * kd[a] + km[a]];",
               "    }", "  } }"]
        return [ind + ln for ln in out]

    # group terms by (a, b) pair
    pairs: Dict[Tuple[int, int], Dict] = {}
    deg1 = []
    for t, (nu, (a, b, c), q) in enumerate(plan.terms):
        if nu == 1:
            deg1.append((t, a, q))
        else:
            g = pairs.setdefault((a, b), {"d2": [], "d3": {}})
            if nu == 2:
                g["d2"].append((t, q))
            else:
                g["d3"].setdefault(c, []).append((t, q))

    head = ["  const int cq = blockIdx.x;", f"  const int n0 = blockIdx.y * {NB};",
            "  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;",
            f"  const int c = __builtin_amdgcn_readfirstlane(cq * {Q} + (wv & {Q - 1}));",
            f"  const int cl = __builtin_amdgcn_readfirstlane(wv & {Q - 1});",
            f"  const int nrow = (wv >> 2) * 64 + lane;      // this lane's node row in the tile",
            f"  const float* __restrict__ cf = coef + (size_t)c * {nt};"]

    # ---------------- forward ----------------
    if not SC_FWD_CP:
        L.append(f"__global__ __launch_bounds__({NTH}) void sc_fwd_{name}(")
        L.append("    const float* __restrict__ x, const float* __restrict__ coef, int n_nodes,")
        L.append("    float* __restrict__ out) {")
        L.append(f"  __shared__ float tile[{NB} * {TP}];")
        L += head
        L += stage_in("x", "tile", lin, NB, NTH)
        L.append("  __syncthreads();")
        # packed: a lane owns nodes n0 + lane and n0 + 64 + lane (one v_pk_* op covers both)
        L.append(f"  float* __restrict__ tr = tile + nrow * {TP};")
        if PKN == 2:
            L.append(f"  float* __restrict__ tr1 = tile + (lane + 64) * {TP};")
        for a in range(D):
            L.append("  " + ld_pair(f"x{a}", "tr", "tr1", lq(lin, a, 'cl')))
        for q in range(Dout):
            L.append(f"  {FT} o{q} = {ZERO};")
        blocks = sc_blocks(plan)
        fv = [f"x{a}" for a in range(D)] + [f"o{q}" for q in range(Dout)]
        for b0 in blocks[:SC_PFD_FWD]:
            for t in b0["terms"]:
                L.append(f"  float c{t} = cf[{t}];")
        for bi, blk in enumerate(blocks):
            # coefficients SC_PFD_FWD blocks ahead are in flight (scalar loads) while this block computes
            for t in (blocks[bi + SC_PFD_FWD]["terms"] if bi + SC_PFD_FWD < len(blocks) else []):
                L.append(f"  float c{t} = cf[{t}];")
            nxt = [t for b1 in blocks[bi + 1: bi + 1 + SC_PFD_FWD] for t in b1["terms"]]
            carry = []
            if blk["kind"] == "deg1":
                for t, a, q in blk["deg1"]:
                    L.append(f"  o{q} = {fma_s(f'c{t}', f'x{a}', f'o{q}')};")
            else:
                a, b = blk["a"], blk["b"]
                pv = f"p{a}_{b}"
                if blk["first"]:
                    L.append(f"  {FT} {pv} = x{a} * x{b};")
                for t, q in blk["d2"]:
                    L.append(f"  o{q} = {fma_s(f'c{t}', pv, f'o{q}')};")
                for cc, lst in blk["d3"]:
                    L.append(f"  {{ const {FT} m = {pv} * x{cc};")
                    for t, q in lst:
                        L.append(f"    o{q} = {fma_s(f'c{t}', 'm', f'o{q}')};")
                    L.append("  }")
                if not blk["last"]:
                    carry = [pv]
            L.append("  " + pin(fv + carry, sgprs=[f"c{t}" for t in nxt]))
        L.append("  __syncthreads();")
        for q in range(Dout):
            L.append("  " + st_pair(f"o{q}", "tr", "tr1", lq(lout, q, 'cl')))
        L.append("  __syncthreads();")
        L += stage_out("out", "tile", lout, NB, NTH)
        L.append("}")

    else:
        # two channels per lane (v_pk_* fp32): a workgroup of 4 waves owns 8 channels x 64
        # nodes; wave w holds channels 2w, 2w+1 of every node in one register pair, and the
        # coefficients come channel-pair interleaved (cf2[t] = {coef[c0][t], coef[c0+1][t]}),
        # one SGPR pair per term
        l8, o8 = Lay(irs, "in8", 8), Lay(out_irs, "out8", 8)
        if o8.comp == l8.comp:
            o8.goff = l8.goff
        T8 = max(l8.QD, o8.QD) + 1
        if T8 % 2 == 0:
            T8 += 1
        for lay in ((l8,) if o8.comp == l8.comp else (l8, o8)):
            L.append(f"__device__ __forceinline__ int {lay.goff}(int q, int cq) {{")
            for (sa, sb, so, sd) in lay.segs[:-1]:
                L.append(f"  if (q < {sb}) return {so} + cq * {8 * sd} + (q - {sa});")
            sa, sb, so, sd = lay.segs[-1]
            L.append(f"  return {so} + cq * {8 * sd} + (q - {sa});")
            L.append("}")

        def st_in8(src, lay):
            per = (64 * lay.QD + 255) // 256
            return ["  { int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));",
                    "#pragma unroll 2",
                    f"  for (int it = 0; it < {per}; ++it) {{",
                    "    const int idx = tid + 256 * it;",
                    f"    if (idx < {64 * lay.QD}) {{",
                    f"      const int nl = idx / {lay.QD}, q = idx - nl * {lay.QD}, n = n0 + nl;",
                    f"      tile[nl * {T8} + q] = (n < n_nodes) ? {src}[(size_t)n * {lay.row} + {lay.goff}(q, cq)] : 0.0f;",
                    "    }", "  } }"]

        def st_out8(dst, lay):
            per = (64 * lay.QD + 255) // 256
            return ["  { int tid = threadIdx.x; asm volatile(\"\" : \"+v\"(tid));",
                    "#pragma unroll 2",
                    f"  for (int it = 0; it < {per}; ++it) {{",
                    "    const int idx = tid + 256 * it;",
                    f"    if (idx < {64 * lay.QD}) {{",
                    f"      const int nl = idx / {lay.QD}, q = idx - nl * {lay.QD}, n = n0 + nl;",
                    f"      if (n < n_nodes) {dst}[(size_t)n * {lay.row} + {lay.goff}(q, cq)] = tile[nl * {T8} + q];",
                    "    }", "  } }"]

        def lq8(lay, a_, cl):
            l_, m_, _, sg = lay.comp[a_]
            return f"{sg} + ({cl}) * {2 * l_ + 1} + {m_}"

        L.append(f"__global__ __launch_bounds__(256) void sc_fwd_{name}(")
        L.append("    const float* __restrict__ x, const float* __restrict__ coef, int n_nodes,")
        L.append("    float* __restrict__ out) {")
        L.append(f"  __shared__ float tile[64 * {T8}];")
        L.append("  const int cq = blockIdx.x;   // channel octet")
        L.append("  const int n0 = blockIdx.y * 64;")
        L.append("  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;")
        L.append("  const int cp = __builtin_amdgcn_readfirstlane(cq * 4 + wv);   // channel pair")
        L.append(f"  const float* __restrict__ cf = coef + (size_t)cp * {2 * nt};")
        L += st_in8("x", l8)
        L.append("  __syncthreads();")
        L.append(f"  float* __restrict__ tr = tile + lane * {T8};")
        for a_ in range(D):
            L.append(f"  eelg_f2 x{a_} = eelg_f2{{tr[{lq8(l8, a_, '2 * wv')}], tr[{lq8(l8, a_, '2 * wv + 1')}]}};")
        for q in range(Dout):
            L.append(f"  eelg_f2 o{q} = eelg_f2{{0.0f, 0.0f}};")
        blocks = sc_blocks(plan, SC_CP_MAXB)
        fv = [f"x{a_}" for a_ in range(D)] + [f"o{q}" for q in range(Dout)]

        def cload(t):
            return f"  eelg_f2 c{t} = *reinterpret_cast<const eelg_f2*>(cf + {2 * t});"
        for b0 in blocks[:SC_PFD_FWD]:
            for t in b0["terms"]:
                L.append(cload(t))
        for bi, blk in enumerate(blocks):
            for t in (blocks[bi + SC_PFD_FWD]["terms"] if bi + SC_PFD_FWD < len(blocks) else []):
                L.append(cload(t))
            nxt = [t for b1 in blocks[bi + 1: bi + 1 + SC_PFD_FWD] for t in b1["terms"]]
            carry = []
            if blk["kind"] == "deg1":
                for t, a_, q in blk["deg1"]:
                    L.append(f"  o{q} = eelg_fma2(c{t}, x{a_}, o{q});")
            else:
                a_, b_ = blk["a"], blk["b"]
                pv = f"p{a_}_{b_}"
                if blk["first"]:
                    L.append(f"  eelg_f2 {pv} = x{a_} * x{b_};")
                for t, q in blk["d2"]:
                    L.append(f"  o{q} = eelg_fma2(c{t}, {pv}, o{q});")
                for cc, lst in blk["d3"]:
                    L.append(f"  {{ const eelg_f2 m = {pv} * x{cc};")
                    for t, q in lst:
                        L.append(f"    o{q} = eelg_fma2(c{t}, m, o{q});")
                    L.append("  }")
                if not blk["last"]:
                    carry = [pv]
            L.append("  " + pin(fv + carry, sgprs=[f"c{t}" for t in nxt]))
        L.append("  __syncthreads();")
        for q in range(Dout):
            L.append(f"  tr[{lq8(o8, q, '2 * wv')}] = o{q}.x; tr[{lq8(o8, q, '2 * wv + 1')}] = o{q}.y;")
        L.append("  __syncthreads();")
        L += st_out8("out", o8)
        L.append("}")

    # ---------------- backward w.r.t. x ----------------
    L.append(f"__global__ __launch_bounds__({NTH}) void sc_bwd_x_{name}(")
    L.append("    const float* __restrict__ x, const float* __restrict__ coef,")
    L.append("    const float* __restrict__ gout, int n_nodes, float* __restrict__ gx,")
    L.append("    float* __restrict__ xt, float* __restrict__ gt) {")
    # one LDS tile, used three times (x in, grad_out in, grad_x out): 2x the occupancy of
    # separate x / grad_out tiles.  When xt / gt are given, the staged tiles are also written
    # channel-major (the coefficient gradient's operands) -- no separate transpose pass.
    L.append(f"  __shared__ float tx[{NB} * {TP}];")
    L += head
    L += stage_in("x", "tx", lin, NB, NTH)
    L.append("  __syncthreads();")
    L.append("  if (xt) {")
    L += cm_store("xt", "tx", lin, NB, "    ", NTH)
    L.append("  }")
    L.append(f"  float* __restrict__ xr = tx + nrow * {TP};")
    if PKN == 2:
        L.append(f"  float* __restrict__ xr1 = tx + (lane + 64) * {TP};")
    for a in range(D):
        L.append("  " + ld_pair(f"x{a}", "xr", "xr1", lq(lin, a, 'cl')))
        L.append(f"  {FT} d{a} = {ZERO};")
    L.append("  __syncthreads();")
    L += stage_in("gout", "tx", lout, NB, NTH)
    L.append("  __syncthreads();")
    L.append("  if (gt) {")
    L += cm_store("gt", "tx", lout, NB, "    ", NTH)
    L.append("  }")
    for q in range(Dout):
        L.append("  " + ld_pair(f"g{q}", "xr", "xr1", lq(lout, q, 'cl')))
    bv = [f"x{a}" for a in range(D)] + [f"g{q}" for q in range(Dout)] + [f"d{a}" for a in range(D)]
    for b0 in blocks[:SC_PFD_BWD]:
        for t in b0["terms"]:
            L.append(f"  float c{t} = cf[{t}];")
    for bi, blk in enumerate(blocks):
        # coefficients SC_PFD_BWD blocks ahead are in flight (scalar loads) while this block computes
        for t in (blocks[bi + SC_PFD_BWD]["terms"] if bi + SC_PFD_BWD < len(blocks) else []):
            L.append(f"  float c{t} = cf[{t}];")
        nxt = [t for b1 in blocks[bi + 1: bi + 1 + SC_PFD_BWD] for t in b1["terms"]]
        carry = []
        if blk["kind"] == "deg1":
            for t, a, q in blk["deg1"]:
                L.append(f"  d{a} = {fma_s(f'c{t}', f'g{q}', f'd{a}')};")
        else:
            a, b = blk["a"], blk["b"]
            pv, sv = f"p{a}_{b}", f"s{a}_{b}"
            if blk["first"]:
                L.append(f"  {FT} {pv} = x{a} * x{b}; {FT} {sv} = {ZERO};")
            for t, q in blk["d2"]:
                L.append(f"  {sv} = {fma_s(f'c{t}', f'g{q}', sv)};")
            for cc, lst in blk["d3"]:
                L.append(f"  {{ {FT} s = {ZERO};")
                for t, q in lst:
                    L.append(f"    s = {fma_s(f'c{t}', f'g{q}', 's')};")
                L.append(f"    d{cc} = {fma_v('s', pv, f'd{cc}')}; {sv} = {fma_v('s', f'x{cc}', sv)}; }}")
            if blk["last"]:
                L.append(f"  d{a} = {fma_v(sv, f'x{b}', f'd{a}')}; d{b} = {fma_v(sv, f'x{a}', f'd{b}')};")
            else:
                carry = [pv, sv]
        L.append("  " + pin(bv + carry, sgprs=[f"c{t}" for t in nxt]))
    L.append("  __syncthreads();")
    for a in range(D):
        L.append("  " + st_pair(f"d{a}", "xr", "xr1", lq(lin, a, 'cl')))
    L.append("  __syncthreads();")
    L += stage_out("gx", "tx", lin, NB, NTH)
    L.append("}")

    # ---------------- mul-major -> channel-major transpose ----------------
    # dst[(c * D + a) * n_nodes + n] = src[n, a-th component of channel c]; one kernel per
    # distinct layout (x uses the input layout, grad_out the output layout)
    def emit_cmajor(kname, lay):
        L.append(f"__global__ __launch_bounds__(256) void {kname}(")
        L.append("    const float* __restrict__ x, int n_nodes, float* __restrict__ xt) {")
        L.append(f"  __shared__ float tile[64 * {TP}];")
        L.append("  const int cq = blockIdx.x;")
        L.append("  const int n0 = blockIdx.y * 64;")
        L.extend(stage_in("x", "tile", lay))
        L.append("  __syncthreads();")
        L.extend(cm_store("xt", "tile", lay, 64))
        L.append("}")
    emit_cmajor(f"sc_cmajor_{name}", lin)
    cmajor_out = f"sc_cmajor_{name}"
    if lout.comp != lin.comp:
        cmajor_out = f"sc_cmajor_out_{name}"
        emit_cmajor(cmajor_out, lout)

    # ---------------- backward w.r.t. coefficients ----------------
    # grad coef[c, t] = sum_n g_q(n) x_a(n) x_b(n) x_c(n).  A workgroup owns one channel and
    # one chunk of SC_COEF_CHUNK nodes: it stages the chunk's channel-major x / g rows into LDS
    # ONCE (every byte of xt / gt crosses HBM once per launch), then its SC_COEF_WAVES waves
    # sweep the staged chunk once per term group (JG accumulators per lane, one lane per node
    # of a 64-node sub-tile) with no further barrier.  The per-lane sums are reduced over the
    # 64 lanes by recursive halving (eelg_lane_reduce64), so lane t ends with term t of the
    # group.  Deterministic partials part[chunk, c, t], summed over chunks by the caller.
    NCB = SC_COEF_CHUNK
    WV = SC_COEF_WAVES
    NPL = SC_COEF_NPL
    gpw = -(-nt // (WV * SC_COEF_MAXJG))      # term groups per wave
    JG = -(-nt // (WV * gpw))                 # terms per group (<= 64)
    assert JG <= 64 and NCB % (64 * NPL) == 0 and NPL in (1, 2)
    groups = [list(range(s, min(s + JG, nt))) for s in range(0, nt, JG)]
    nsub = NCB // (64 * NPL)
    NC4 = NCB // 4
    L.append(f"// coefficient gradient: {len(groups)} term groups of <= {JG} terms, {gpw} per wave;")
    L.append(f"// one workgroup = one channel x {NCB} LDS-resident nodes")
    L.append(f"__global__ __launch_bounds__({64 * WV}) void sc_bwd_coef_{name}(")
    L.append("    const float* __restrict__ xt, const float* __restrict__ gt, int n_nodes, int chunk,")
    L.append("    float* __restrict__ part) {")
    if SC_COEF_MULMAJOR:
        # operands read straight from the mul-major rows x[N, drow] / grad_out[N, orow] (no
        # channel-major copies): the MUL channel workgroups of one chunk are dispatched back to
        # back on one XCD (block id % 8), so the chunk's rows (NCB x (drow + orow) floats) are
        # fetched from HBM once and served to the 32 channels from that XCD's L2
        SXS = NCB + 1                          # odd stride: the staging stores spread over banks
        lays = [(lin, "xt", drow), (lout, "gt", orow)]
        offs = [lay.comp[a][2] for lay, _, _ in lays for a in range(lay.D)]
        dims = [2 * lay.comp[a][0] + 1 for lay, _, _ in lays for a in range(lay.D)]
        ms = [lay.comp[a][1] for lay, _, _ in lays for a in range(lay.D)]
        L.append(f"  __shared__ float sx[{D} * {SXS}];")
        L.append(f"  __shared__ float sg[{Dout} * {SXS}];")
        L.append("  const int id = blockIdx.x, xcd = id & 7, rest = id >> 3;")
        L.append(f"  const int c = rest % {MUL}, ch = (rest / {MUL}) * 8 + xcd;")
        L.append(f"  const int nb = ch * {NCB};")
        L.append("  if (nb >= n_nodes) return;   // uniform per workgroup")
        L.append(f"  const int koff[{D + Dout}] = {{{', '.join(str(o + m) for o, m in zip(offs, ms))}}};")
        L.append(f"  const int kd[{D + Dout}] = {{{', '.join(str(d) for d in dims)}}};")
        L.append(f"  for (int i = threadIdx.x; i < {(D + Dout) * NCB}; i += {64 * WV}) {{")
        L.append(f"    const int j = i / {D + Dout}, a = i - j * {D + Dout};")
        L.append("    const int n = nb + j;")
        L.append(f"    const bool isx = a < {D};")
        L.append(f"    const float* __restrict__ row = isx ? xt + (size_t)n * {drow} : gt + (size_t)n * {orow};")
        L.append("    const float v = n < n_nodes ? row[koff[a] + c * kd[a]] : 0.0f;")
        L.append(f"    (isx ? sx + a * {SXS} : sg + (a - {D}) * {SXS})[j] = v;")
        L.append("  }")
    else:
        SXS = NCB
        L.append(f"  __shared__ float sx[{D} * {NCB}];")
        L.append(f"  __shared__ float sg[{Dout} * {NCB}];")
        L.append("  const int ch = blockIdx.x, c = blockIdx.y;")
        L.append(f"  const int nb = ch * {NCB};")
        L.append(f"  const int cnt = min({NCB}, n_nodes - nb);")
        L.append("  const bool vec = (n_nodes & 3) == 0;")
        L.append(f"  for (int i = threadIdx.x; i < {(D + Dout) * NC4}; i += {64 * WV}) {{")
        L.append(f"    const int a = i / {NC4}, j = 4 * (i - a * {NC4});")
        L.append(f"    const float* __restrict__ src = a < {D} ? xt + ((size_t)c * {D} + a) * n_nodes"
                 f" : gt + ((size_t)c * {Dout} + (a - {D})) * n_nodes;")
        L.append(f"    float* __restrict__ sdst = a < {D} ? sx + a * {NCB} + j : sg + (a - {D}) * {NCB} + j;")
        L.append("    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);")
        L.append("    if (vec && j + 4 <= cnt) {")
        L.append("      v = *reinterpret_cast<const float4*>(src + nb + j);")
        L.append("    } else {")
        L.append("      if (j + 0 < cnt) v.x = src[nb + j + 0];")
        L.append("      if (j + 1 < cnt) v.y = src[nb + j + 1];")
        L.append("      if (j + 2 < cnt) v.z = src[nb + j + 2];")
        L.append("      if (j + 3 < cnt) v.w = src[nb + j + 3];")
        L.append("    }")
        L.append("    *reinterpret_cast<float4*>(sdst) = v;")
        L.append("  }")
    L.append("  __syncthreads();")
    L.append("  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;")
    L.append(f"  float* __restrict__ dst = part + ((size_t)ch * {MUL} + c) * {nt};")
    L.append(f"  for (int k = 0; k < {gpw}; ++k) {{")
    L.append(f"    const int jg = __builtin_amdgcn_readfirstlane(k * {WV} + wv);")
    L.append("    float acc[64];")
    L.append("#pragma unroll")
    L.append("    for (int i = 0; i < 64; ++i) acc[i] = 0.0f;")
    L.append("    switch (jg) {")
    for gi, grp in enumerate(groups):
        L.append(f"    case {gi}: {{")
        need_x, need_g = set(), set()
        for t in grp:
            nu, (a, b, cc), q = plan.terms[t]
            need_g.add(q)
            need_x.add(a)
            if nu >= 2:
                need_x.add(b)
            if nu >= 3:
                need_x.add(cc)
        cpin = pin([f"acc[{jj}]" for jj in range(len(grp))])
        L.append(f"#pragma unroll {SC_COEF_UNROLL}")
        L.append(f"      for (int sb = 0; sb < {nsub}; ++sb) {{")
        L.append(f"        const int o = sb * {64 * NPL} + {NPL} * lane;")
        if NPL == 1:
            for a in sorted(need_x):
                L.append(f"        const float x{a} = sx[{a * SXS} + o];")
            for q in sorted(need_g):
                L.append(f"        const float g{q} = sg[{q * SXS} + o];")
            halves = [""]
        else:
            # adjacent nodes o, o + 1 of one operand in one 8-byte read; the terms run per node
            for a in sorted(need_x):
                L.append(f"        const float2 x{a} = *reinterpret_cast<const float2*>(&sx[{a * SXS} + o]);")
            for q in sorted(need_g):
                L.append(f"        const float2 g{q} = *reinterpret_cast<const float2*>(&sg[{q * SXS} + o]);")
            halves = [".x", ".y"]
        for h in halves:
            cur = None
            for jj, t in enumerate(grp):
                nu, (a, b, cc), q = plan.terms[t]
                if nu == 1:
                    L.append(f"        acc[{jj}] = fmaf(x{a}{h}, g{q}{h}, acc[{jj}]);")
                    continue
                if cur != (a, b):
                    if cur is not None:
                        L.append("        }")
                        L.append("        " + cpin)
                    L.append(f"        {{ const float p = x{a}{h} * x{b}{h};")
                    cur = (a, b)
                if nu == 2:
                    L.append(f"          acc[{jj}] = fmaf(p, g{q}{h}, acc[{jj}]);")
                else:
                    L.append(f"          acc[{jj}] = fmaf(p * x{cc}{h}, g{q}{h}, acc[{jj}]);")
            if cur is not None:
                L.append("        }")
            L.append("        " + cpin)
        L.append("      }")
        L.append("      break; }")
    L.append("    default: break;")
    L.append("    }")
    L.append("    eelg_lane_reduce64(acc);")
    L.append(f"    const int t = jg * {JG} + lane;")
    L.append(f"    if (jg < {len(groups)} && lane < {JG} && t < {nt}) dst[t] = acc[0];")
    L.append("  }")
    L.append("}")
    WPB, NBC = WV, NCB
    info = dict(D=D, Dout=Dout, drow=drow, orow=orow, nterms=nt, njg=len(groups), wpb=WPB, nb=NB, nbc=NBC, nth=NTH,
                coef_mulmajor=SC_COEF_MULMAJOR, fwd_cp=SC_FWD_CP,
                cmajor_out=cmajor_out, sig=fnv1a64(sc_signature(coupling, ls, corr)))
    return "\n".join(L), info


# ---------------------------------------------------------------------------
def main(outdir: str) -> None:
    os.makedirs(outdir, exist_ok=True)
    parts = ["// GENERATED by csrc/gen_kernels.py -- do not edit", "#include <hip/hip_runtime.h>",
             "#include <stdint.h>", '#include "../eelg_internal.h"', "",
             "// dword-aligned vector types: per-lane runs of d floats start at 4-byte boundaries",
             "typedef float eelg_f4u __attribute__((ext_vector_type(4), aligned(4)));",
             "typedef float eelg_f3u __attribute__((ext_vector_type(3), aligned(4)));",
             "typedef float eelg_f2u __attribute__((ext_vector_type(2), aligned(4)));",
             "typedef float eelg_f4a __attribute__((ext_vector_type(4)));",
             "// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two fp32 lanes per instruction)",
             "typedef float eelg_f2 __attribute__((ext_vector_type(2)));",
             "__device__ __forceinline__ eelg_f2 eelg_fma2(eelg_f2 a, eelg_f2 b, eelg_f2 c) {"
             " return __builtin_elementwise_fma(a, b, c); }",
             "__device__ __forceinline__ eelg_f2 eelg_fma2s(float a, eelg_f2 b, eelg_f2 c) {"
             " return __builtin_elementwise_fma(eelg_f2{a, a}, b, c); }",
             "// two nodes per lane in plain fp32 (EELG_SC_PK=3): a struct, so no packed ops form",
             "struct eelg_d2 { float x, y; };",
             "__device__ __forceinline__ eelg_d2 operator*(eelg_d2 a, eelg_d2 b) { return {a.x * b.x, a.y * b.y}; }",
             "__device__ __forceinline__ eelg_d2 eelg_fma2(eelg_d2 a, eelg_d2 b, eelg_d2 c) {"
             " return {fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }",
             "__device__ __forceinline__ eelg_d2 eelg_fma2s(float a, eelg_d2 b, eelg_d2 c) {"
             " return {fmaf(a, b.x, c.x), fmaf(a, b.y, c.y)}; }", ""]
    for lmax in kernel_sets.LMAX:
        parts.append(emit_sh(lmax))
    tp_table, sc_table = [], []
    for name, (node, sh, target) in tp_configs().items():
        code, info = emit_tp(name, node, sh, target)
        parts.append(code)
        parts.append(emit_tp(name, node, sh, target, "bf16")[0])
        tp_table.append((name, info))
    for name, (coupling, ls, corr) in sc_configs().items():
        code, info = emit_sc(name, coupling, ls, corr)
        parts.append(code)
        sc_table.append((name, info))
    # launch tables
    parts.append("\n// ===== config tables =====")
    parts.append("static const eelg_tp_cfg kTpConfigs[] = {")
    for name, i in tp_table:
        lmax = int(name.split("_l")[1])
        parts.append(f'  {{"{name}", {i["din"]}, {i["dmid"]}, {i["wn"]}, {i["nsh"]}, {i["ngroups"]}, '
                     f'{i["npaths"]}, {lmax}, {i["nbgroups"]}, {i["nph"]}, {i["beph"]}, 0x{i["sig"]:016x}ULL, tp_fwd_{name}, tp_bwd_{name}, '
                     f'tp_fwd_{name}_bw, tp_bwd_{name}_bw, tp_bws_{name}, tp_bws_{name}_bw, '
                     f'{i["fwd_threads"]}, {i["fwd_tile"]}}},')
    parts.append("};")
    parts.append("static const eelg_sc_cfg kScConfigs[] = {")
    for name, i in sc_table:
        parts.append(f'  {{"{name}", {i["D"]}, {i["Dout"]}, {i["drow"]}, {i["orow"]}, {i["nterms"]}, {i["njg"]}, {i["wpb"]}, '
                     f'0x{i["sig"]:016x}ULL, sc_fwd_{name}, sc_bwd_x_{name}, sc_bwd_coef_{name}, sc_cmajor_{name}, '
                     f'{i["cmajor_out"]}, {i["nb"]}, {i["nbc"]}, {i["coef_mulmajor"]}, {i["fwd_cp"]}, {i["nth"]}}},')
    parts.append("};")
    parts.append("const eelg_tp_cfg* eelg_tp_table(int* n) { *n = (int)(sizeof(kTpConfigs)/sizeof(kTpConfigs[0])); return kTpConfigs; }")
    parts.append("const eelg_sc_cfg* eelg_sc_table(int* n) { *n = (int)(sizeof(kScConfigs)/sizeof(kScConfigs[0])); return kScConfigs; }")
    src = "\n".join(parts) + "\n"
    path = os.path.join(outdir, "eelg_gen.hip")
    old = open(path).read() if os.path.exists(path) else None
    if old != src:
        with open(path, "w") as f:
            f.write(src)
    print(f"wrote {path}: {len(src.splitlines())} lines")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "generated"))
