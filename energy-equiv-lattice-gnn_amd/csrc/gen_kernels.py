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
# measurement variant (never the product): tp_fwd computes every aggregate but stores none, the
# lower bound of a forward that hands agg to a fused epilogue instead of HBM
TP_FWD_NOSTORE = int(os.environ.get("EELG_TP_FWD_NOSTORE", "0"))
TP_MAXACC = int(os.environ.get("EELG_TP_MAXACC", "64"))
# the bf16-weight forward's path groups (config 5): smaller groups, 109 instead of 141 VGPRs.
# r06d / r06e (lmax 3, 5k-node lattices): tp_fwd_tpB_l3_bw 0.477 -> 0.4985 of the roof; at 64
# for fp32 (config 2: a cap of 40 took tp_fwd from 0.54 to 0.48, r06f)
TP_MAXACC_BF = int(os.environ.get("EELG_TP_MAXACC_BF", "40"))
# tp_fwd waves per workgroup (a node tile = 2 x TP_FWD_WPB x TP_NPH receivers; one-wave
# workgroups refill a freed wave slot at once: r03z kbench 0.505 vs 0.520 ms at 4, 0.518 at 2;
# in the step 0.438 vs 0.446 ms)
TP_FWD_WPB = int(os.environ.get("EELG_TP_FWD_WPB", "1"))
# tp_fwd: the rows of the next two edges (x / SH / weight) prefetched into LDS by LDS-DMA
# (global_load_lds) instead of a second register set, for fp32 and bf16 weight storage.  One
# edge in flight by LDS-DMA (r03ag/r03ai: 0.499 vs 0.486 ms kbench) and the register pipeline
# (0.513 ms; 0.439 vs 0.418 ms in the step) were removed.
# LDS-DMA tp_fwd: minimum waves per SIMD asked of the register allocator (0: none)
TP_FWD_WPE = int(os.environ.get("EELG_TP_FWD_WPE", "0"))
# LDS-DMA tp_fwd: a group's weight slices lead its chunk list, and the LDS-DMA instructions that
# move only weights carry the nontemporal cache policy (the 705 MB weight stream is read once;
# the x rows gathered per in-edge stay cacheable).  r04t: in the step 0.418 -> 0.410 ms per launch
# (roofline 0.535 -> 0.545), kbench 0.500 -> 0.492 ms; the step unchanged
TP_FWD_WNT = int(os.environ.get("EELG_TP_FWD_WNT", "1"))
# LDS-DMA tp_fwd: the aggregate rows stored nontemporal (r03l/r03n with the register pipeline:
# the kernel 3 % faster, the step 0.4 % slower as the following linear missed in L2; r04w: kbench
# 0.491 -> 0.469 ms, but in the step the kernel itself 0.406 -> 0.418 ms and the step equal)
TP_FWD_ANT = int(os.environ.get("EELG_TP_FWD_ANT", "0"))
# LDS-DMA tp_fwd: edges in flight per half-wave (LDS image buffers), fp32 / bf16 weight storage
TP_FWD_NBUF = int(os.environ.get("EELG_TP_FWD_NBUF", "2"))
TP_FWD_NBUF_BF = int(os.environ.get("EELG_TP_FWD_NBUF_BF", "2"))

TP_BWD_EPH = int(os.environ.get("EELG_TP_BWD_EPH", "1"))   # edges per half-wave in tp_bwd (4: 0.88 ms, 8: 0.90 ms vs 0.76 ms at 1)
# tp_bwd: paths whose grad_agg slice + weight are in flight ahead of the path being computed
# (r03v: 1: 0.781 ms, 2: 0.713, 3: 0.727)
TP_BWD_PFD = int(os.environ.get("EELG_TP_BWD_PFD", "2"))
# tp_bwd (fp32): grad_w and gxe stored nontemporal (read back by later kernels: the sender sum,
# the radial MLP backward on its side stream).  r04r: kbench 0.701 -> 0.683 ms, step +0.3-0.4 %
TP_BWD_NT = int(os.environ.get("EELG_TP_BWD_NT", "1"))
# tp_bwd block placement: 0 = 2-D grid (edge block, input-block group), consecutive edge blocks
# dealt round-robin over the 8 XCDs; 1 = 1-D grid, XCD k takes one contiguous range of edge
# blocks with the groups of an edge block adjacent; 2 = the same ranges, group-major per XCD.
# With 0 a receiver whose in-edges straddle two blocks has its grad_agg row fetched into two
# L2s, and every XCD gathers every lattice's x rows
TP_BWD_XCD = int(os.environ.get("EELG_TP_BWD_XCD", "2"))
# tp_bwd: amdgpu_waves_per_eu floor (0: the compiler's 125 VGPRs, 4 waves / SIMD).  Round 6: 5
# spills 87 VGPRs of tpB_l4 to scratch, 6 spills 303 -- the l4 kernel has no occupancy lever
TP_BWD_WPE = int(os.environ.get("EELG_TP_BWD_WPE", "0"))
# fused output-linear grad-x + TP backward (tp_bwf, mul 32; off by default, gnn/ops.py TP_BWF):
# receivers per workgroup whose [Σ d3 × 32] grad_agg block of one input-block group is computed
# by MFMA into LDS from the linear's output gradient, then read by the tile's in-edges.
# r09c kbench (tp_bwd 0.682 + linear grad-x 0.324 ms unfused): R 8 receiver-major 1.417 ms,
# edge-major 1.242, edge-major without the next-edge prefetch 1.142, the same at R 4 1.104;
# the MFMA stage alone (R 8) 0.505 ms -- latency-bound at 2 waves / SIMD (LDS and VGPRs)
TP_BWF_R = int(os.environ.get("EELG_TP_BWF_R", "4"))
TP_BWF_SKIP = int(os.environ.get("EELG_TP_BWF_SKIP", "0"))   # measurement only: 1 = no edge stage, 2 = no MFMA stage
TP_BWF_EM = int(os.environ.get("EELG_TP_BWF_EM", "1"))       # edge stage: 1 = the tile's edges dealt over the half-waves
TP_BWF_NX = int(os.environ.get("EELG_TP_BWF_NX", "0"))       # edge stage: next edge's x / SH / weight loads one edge ahead
TP_BWF_P1PF = int(os.environ.get("EELG_TP_BWF_P1PF", "1"))   # MFMA stage: next task's operands loaded one task ahead
# symmetric contraction: coefficient blocks (32 terms each) in flight ahead of the block being
# computed, and the terms per block, forward / grad-x (r03r/r03s, grad-x: 32 terms 2 ahead
# 0.407 ms, 64 terms 1 ahead 0.363 ms; 16 terms 3-4 ahead 0.57 ms; the forward: 32 or 40 terms
# 1 ahead, it spills SGPRs beyond)
SC_PFD_FWD = int(os.environ.get("EELG_SC_PFD_FWD", "1"))
SC_BLOCK_FWD = int(os.environ.get("EELG_SC_BLOCK_FWD", "32"))
SC_PFD_BWD = int(os.environ.get("EELG_SC_PFD_BWD", "1"))
SC_BLOCK_BWD = int(os.environ.get("EELG_SC_BLOCK_BWD", "64"))
# fwd / grad-x: 64-node tiles per workgroup; waves w, w + 4, ... run the same channel on
# consecutive tiles, so their coefficient scalar loads share the CU's scalar cache
SC_NT = int(os.environ.get("EELG_SC_NT", "1"))
# fwd / grad-x: a block's coefficients are scalar-loaded as SGPR vectors (16 / 8 / 4 / 2 / 1
# terms per s_load) and pinned as whole vectors, so the VALU reads them in place; 0 = one float
# (and one pinned SGPR, hence an s_mov_b32 per term) per coefficient.  r04f kbench: fwd 0.312 vs
# 0.326 ms, grad-x 0.349 vs 0.357
SC_CVEC = int(os.environ.get("EELG_SC_CVEC", "1"))
# fwd / grad-x packed: two nodes per lane (lane, lane + 64 of a 128-node tile) on v_pk_fma_f32,
# each coefficient broadcast from ONE half of an aligned SGPR pair by op_sel / op_sel_hi (inline
# asm: the compiler builds (c, c) pairs with an s_mov per odd coefficient instead).  Round-5
# microbenchmark (tools/proto/valu_ceiling.hip, profiles/r05b_valu.txt): a plain v_fmac_f32 with
# an SGPR operand issues once per ~4 cycles per SIMD at ANY occupancy (77 TFLOP/s), all-VGPR
# FMAs reach 118-120 TF and the op_sel-broadcast packed FMA 132-140 TF at 2-4 waves per SIMD
SC_PK = int(os.environ.get("EELG_SC_PK", "1"))
# packed grad-x: 32-term blocks (64 with one block ahead spills SGPRs once the volatile packed
# statements fix the order)
SC_PK_BLOCK_BWD = int(os.environ.get("EELG_SC_PK_BLOCK_BWD", "32"))
# packed: 1 = every packed statement a volatile asm in the _PkSched order; 0 = the broadcast FMAs
# as plain asm and the VGPR products / FMAs as vector C++, in term order, scheduled by the compiler
SC_PK_SCHED = int(os.environ.get("EELG_SC_PK_SCHED", "1"))
# packed coefficient operands: "asm" = one aligned SGPR pair per two terms, the odd term broadcast
# by op_sel in inline asm; "dual" = each block scalar-loaded twice (at t0 and t0 + 1), so every
# coefficient is the LOW half of an aligned pair, which the compiler broadcasts by itself
# (op_sel_hi:[0,..]) -- no inline asm, no hazard s_nops, twice the SGPRs per block
SC_PK_MODE = os.environ.get("EELG_SC_PK_MODE", "asm")
# coefficient gradient: LDS-resident nodes per workgroup, waves per workgroup, the most
# accumulators (terms) per wave
SC_COEF_CHUNK = int(os.environ.get("EELG_SC_COEF_CHUNK", "512"))
SC_COEF_WAVES = int(os.environ.get("EELG_SC_COEF_WAVES", "16"))
SC_COEF_MAXJG = int(os.environ.get("EELG_SC_COEF_MAXJG", "64"))
# coefficient gradient: term groups clustered by shared operands (coef_groups) instead of runs
# of the term order
SC_COEF_CLUSTER = int(os.environ.get("EELG_SC_COEF_CLUSTER", "1"))
# coefficient gradient, streaming form (round 6): a wave owns ONE term group for a whole node
# range, so its accumulators are zeroed and reduced across the lanes once per range instead of
# once per 512-node chunk (the round-5 form spent ~21 % of its VALU instructions there); the
# range's channel-major rows stream through two LDS buffers of SC_COEF_SC nodes filled by
# LDS-DMA one chunk ahead.  0 = the round-5 chunk-resident kernel
SC_COEF_STREAM = int(os.environ.get("EELG_SC_COEF_STREAM", "1"))
SC_COEF_SC = 256                      # nodes per streamed chunk: one 1-KiB LDS-DMA row per wave-instruction
# streamed image as row pairs read by ds_read_b64 (1), or as rows read by ds_read2st64_b32 (0).
# Measured (kbench, same boxes): rows 0.402-0.404 ms; pairs 0.578 ms (r08f, the DMA issue loop
# with per-instruction divisions) and 0.464 ms (r08g, strength-reduced issue: 208 four-byte
# LDS-DMA instructions per chunk instead of 50 sixteen-byte ones, SALU 55 -> 88 M, issue
# stalls 186 -> 260 M per launch) -- the halved LDS read cycles do not pay for the fill
SC_COEF_PAIRS = int(os.environ.get("EELG_SC_COEF_PAIRS", "0"))
# packed streaming coefficient gradient: two nodes per lane (a ds_read_b64 of two consecutive
# nodes of a row), v_pk_mul_f32 / v_pk_fma_f32 on node pairs, <= SC_COEF_PK_JG terms per group
# (two accumulator registers per term).  Measured (r08i, kbench): 0.500-0.506 vs 0.410 ms
# unpacked -- VALU instructions 208 -> 129 M per launch, but the 32-term groups need 15 sets
# of workgroups per tile (twice the chunk staging) and a step's compute shrinks 3.5x against a
# fixed staging and barrier cost (SQ_WAIT_ANY 42 %), so it stays off
SC_COEF_PK = int(os.environ.get("EELG_SC_COEF_PK", "0"))
SC_COEF_PK_JG = int(os.environ.get("EELG_SC_COEF_PK_JG", "32"))
# Variants built, measured slower and removed (DESIGN.md section 3 records the numbers): packed
# channel-pair TP forward, 2x-unrolled TP edge loop, shared-coupling (M in LDS) and cooperative
# TP forwards, two nodes / two channels per lane in the contraction, mul-major coefficient
# gradient operands, two node tiles per contraction workgroup.

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
        assert str(target) == kernel_sets.coupling_target(lmax, MUL)
        out[f"tpA_l{lmax}"] = (Irreps(f"{MUL}x0e"), sh, target)
        out[f"tpB_l{lmax}"] = (hidden_irreps(lmax, MUL), sh, target)
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


def vec_store(vals: Sequence[str], base: str, start: str, nt: bool = False) -> List[str]:
    """base[start + i] = vals[i] with dword-aligned 4/3/2-wide stores (nontemporal when nt)"""
    out, i = [], 0
    while i < len(vals):
        w = min(4, len(vals) - i)
        if w == 1:
            out.append(f"__builtin_nontemporal_store({vals[i]}, &{base}[{start} + {i}]);" if nt
                       else f"{base}[{start} + {i}] = {vals[i]};")
        elif nt:
            out.append(f"__builtin_nontemporal_store({_VT[w]}{{" + ", ".join(vals[i: i + w])
                       + f"}}, reinterpret_cast<{_VT[w]}*>({base} + {start} + {i}));")
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


def _chan_groups():
    """(channel groups, lanes per group) of the interaction kernels: a half-wave computes 32
    channels of one receiver / edge, so mul = 64 runs as two channel groups and mul = 16 as one
    group whose lanes 16..31 compute nothing that is stored"""
    return max(1, MUL // 32), min(MUL, 32)


def _glds_chunks(groups, nshp, node_off, wes: int = 4, cg: int = 0):
    """Per path group: the 16-B chunk list of one half-wave's rows for one edge (x blocks of
    x[sender], the SH row, the group's weight slices of ``wes`` bytes per weight) and the image
    offsets in 4-byte units; ``cg`` = the channel group (its lanes' channel slice of every row)."""
    _, LW = _chan_groups()
    glist = []
    for grp in groups:
        need_l1 = sorted({p.l1 for p in grp})
        need_l2 = sorted({p.l2 for p in grp})
        chunks, fo_x, fo_w = [], {}, {}

        def add_w():
            for p in grp:
                fo_w[p.slot] = 4 * len(chunks)
                chunks.extend((2, wes * (p.slot * MUL + cg * LW) + 16 * cc) for cc in range(wes * LW // 16))
        if TP_FWD_WNT:
            add_w()
        for l in need_l1:
            fo_x[l] = 4 * len(chunks)
            chunks += [(0, 4 * (node_off[l] + cg * LW * (2 * l + 1)) + 16 * cc) for cc in range(LW * (2 * l + 1) // 4)]
        fo_sh = 4 * len(chunks)
        chunks += [(1, 16 * cc) for cc in range(nshp // 4)]
        if not TP_FWD_WNT:
            add_w()
        glist.append((need_l1, need_l2, chunks, fo_x, fo_sh, fo_w))
    return glist


def _glds_desc(chunks, nj) -> List[str]:
    """per-lane chunk descriptors (loop-invariant): chunk 64 j + lane = (row kind, byte offset)"""
    out = []
    for j in range(nj):
        runs = []
        for c in range(64 * j, min(64 * j + 64, len(chunks))):
            k, o = chunks[c]
            if runs and runs[-1][2] == k and runs[-1][3] + 16 * (c - runs[-1][0]) == o and runs[-1][1] == c:
                runs[-1][1] = c + 1
            else:
                runs.append([c, c + 1, k, o])
        kexpr, oexpr = "1", "0"             # past the list: chunk 0 of the SH row (discarded)
        for a, b, k, o in reversed(runs):
            kexpr = f"(c_ < {b} ? {k} : {kexpr})"
            oexpr = f"(c_ < {b} ? {o} + 16 * (c_ - {a}) : {oexpr})"
        out.append(f"    int kd{j}, of{j}; {{ const int c_ = {64 * j} + lane; kd{j} = {kexpr}; of{j} = {oexpr}; }}")
    return out


def _glds_compute(grp, cur, accs) -> List[str]:
    """edge e's contribution of one path group, from the registers in ``cur``"""
    L = []
    cpin = pin(accs + cur)
    xn = lambda p, i: f"x{p.l1}_{i}"  # noqa: E731
    yn = lambda p, j: f"y{p.l2 * p.l2 + j}"  # noqa: E731
    for p in grp:
        d1, d2, d3 = 2 * p.l1 + 1, 2 * p.l2 + 1, 2 * p.l3 + 1
        L.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
        L.append(f"        const float wp = w{p.slot} * ({flit(p.coef)} * inv_norm);")
        fold = min((d3 + 1, "none"), (d1, "x"), (d2, "y"))
        if fold[1] == "none":
            _emit_t(p, xn, yn, "t", L, "        ")
            for k in range(d3):
                L.append(f"        a{p.slot}_{k} = fmaf(wp, t{k}, a{p.slot}_{k});")
        else:
            if fold[1] == "x":
                for i in range(d1):
                    L.append(f"        const float xw{i} = {xn(p, i)} * wp;")
                xf, yf = (lambda p, i: f"xw{i}"), yn
            else:
                for j in range(d2):
                    L.append(f"        const float yw{j} = {yn(p, j)} * wp;")
                xf, yf = xn, (lambda p, j: f"yw{j}")
            _emit_acc(p, xf, yf, lambda k, p=p: f"a{p.slot}_{k}", L, "        ")
        L.append("      }")
        L.append("      " + cpin)
    return L


def _emit_tp_fwd_glds2(name, groups, din, nshp, dmid, wn, node_off, bf: bool = False) -> List[str]:
    """tp_fwd with the rows of edges e+1 AND e+2 in flight by LDS-DMA (two LDS images per
    half-wave) while edge e computes.  The per-half-wave stream state (edge, receiver, the
    rowptr entries, the sender indices) is wave-uniform per half and kept in SGPRs with scalar
    loads, so the loop issues no vector load besides the LDS-DMA ones and a counted
    ``s_waitcnt vmcnt(N)`` (N = the LDS-DMA instructions of one edge) retires edge e+1's rows
    while edge e+2's stay in flight.  Stores of a half-wave's aggregates are exec-masked to
    its lanes."""
    WPB = TP_FWD_WPB
    TN = 2 * WPB * TP_NPH
    NBUF = TP_FWD_NBUF_BF if bf else TP_FWD_NBUF
    assert NBUF >= 2
    CG, LW = _chan_groups()
    ng = len(groups) * CG                 # blocks per node tile: (path group, channel group)
    glists = [_glds_chunks(groups, nshp, node_off, 2 if bf else 4, c) for c in range(CG)]
    NJ = max(-(-len(g[2]) // 64) for gl in glists for g in gl)
    NI = NJ * 64
    L: List[str] = []
    wpe = f" __attribute__((amdgpu_waves_per_eu({TP_FWD_WPE})))" if TP_FWD_WPE else ""
    WT = "unsigned short" if bf else "float"
    L.append(f"__global__ __launch_bounds__({64 * WPB}){wpe} void tp_fwd_{name}{'_bw' if bf else ''}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ rowptr, int n_nodes,")
    L.append("    float inv_norm, float* __restrict__ agg) {")
    L.append(f"  __shared__ float4 img_[{WPB}][{NBUF}][2][{NI}];   // [wave][buffer][half][chunk]")
    L.append("  const int lane = threadIdx.x & 63, hf = lane >> 5;")
    L.append("  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
    L.append("  const int u = lane & 31;")
    L.append(f"  const int ntl = (n_nodes + {TN - 1}) / {TN}, tpx = (ntl + 7) >> 3;")
    L.append(f"  const int q = blockIdx.x >> 3, grp = q % {ng};")
    L.append(f"  const int tile = (blockIdx.x & 7) * tpx + q / {ng};")
    L.append(f"  const int nw0 = (tile * {WPB} + wv) * {2 * TP_NPH};")
    L.append("  if (nw0 >= n_nodes) return;   // uniform per wave; a half past the end gets no receivers")
    L.append("  float4* __restrict__ ib = &img_[wv][0][0][0];")
    L.append("  const char* pad_ = reinterpret_cast<const char*>(eelg_tp_pad);")
    L.append("  const unsigned lds0 = (unsigned)(size_t)((__attribute__((address_space(3))) float4*)ib);")
    for h in (0, 1):
        L.append(f"  const int n0_{h} = min(nw0 + {h * TP_NPH}, n_nodes), n1_{h} = min(n0_{h} + {TP_NPH}, n_nodes);")
        L.append(f"  int e_{h} = rowptr[n0_{h}];")
        L.append(f"  const int eend_{h} = rowptr[n1_{h}];")
        L.append(f"  int node_{h} = n0_{h}, nend_{h} = rowptr[min(n0_{h} + 1, n1_{h})], "
                 f"nend2_{h} = rowptr[min(n0_{h} + 2, n1_{h})];")
    L.append("  switch (grp) {")
    for ci, (gi, cg) in enumerate((gi, cg) for gi in range(len(groups)) for cg in range(CG)):
        grp = groups[gi]
        need_l1, need_l2, chunks, fo_x, fo_sh, fo_w = glists[cg][gi]
        nj = -(-len(chunks) // 64)
        L.append(f"  case {ci}: {{ // {len(chunks)} chunks of 16 B per half-wave and edge"
                 + (f", channel group {cg}" if CG > 1 else ""))
        L += _glds_desc(chunks, nj)

        def issue(buf, ahead):
            out = ["    {"]
            for h in (0, 1):
                # a half past its last edge reads the pad row (no edge row need exist: E = 0)
                out.append(f"      {{ const bool ok_ = e_{h} + {ahead} < eend_{h};")
                out.append(f"        const int ee_ = ok_ ? e_{h} + {ahead} : 0;")
                out.append(f"        const int ss_ = *(ok_ ? sender + ee_ : reinterpret_cast<const int*>(pad_));   // never a load through a null sender (E = 0)")
                out.append(f"        const char* xb = ok_ ? reinterpret_cast<const char*>(x + (size_t)ss_ * {din}) : pad_;")
                out.append(f"        const char* shb = ok_ ? reinterpret_cast<const char*>(sh + (size_t)ee_ * {nshp}) : pad_;")
                out.append(f"        const char* wb = ok_ ? reinterpret_cast<const char*>(w + (size_t)ee_ * {wn}) : pad_;")
                out.append(f"        float4* dst = ib + ({buf}) * {2 * NI} + {h * NI};")
                for j in range(nj):
                    # cache policy 2 = nt on gfx950: an instruction that moves only weight chunks
                    only_w = TP_FWD_WNT and all(k == 2 for k, _ in chunks[64 * j: 64 * j + 64])
                    out.append(f"        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)"
                               f"((kd{j} == 0 ? xb : kd{j} == 1 ? shb : wb) + of{j}), "
                               f"(__attribute__((address_space(3))) void*)(dst + {64 * j}), 16, 0, {2 if only_w else 0});")
                out.append("      }")
            out.append("    }")
            return out
        accs = [f"a{p.slot}_{k}" for p in grp for k in range(2 * p.l3 + 1)]
        cur = ([f"x{l}_{i}" for l in need_l1 for i in range(2 * l + 1)]
               + [f"y{l * l + j}" for l in need_l2 for j in range(2 * l + 1)]
               + [f"w{p.slot}" for p in grp])
        L.append("    float " + ", ".join(f"{a} = 0.0f" for a in accs) + ";")
        for k in range(NBUF):
            L += issue(str(k), k)
        L.append("    int b = 0;")
        L.append("    for (;;) {")
        # edge e's rows: everything but the later edges' LDS-DMA instructions has landed
        L.append(f'      asm volatile("s_waitcnt vmcnt({(NBUF - 1) * 2 * nj})" ::: "memory");')
        # the LDS reads are inline asm: hipcc would otherwise order every LDS read after ALL
        # outstanding LDS-DMA (a vmcnt(0): it cannot tell the image being read from the one
        # being filled), which would retire edge e+2's rows too
        L.append(f"      const unsigned imb = lds0 + b * {2 * NI * 16} + hf * {NI * 16};")
        L.append("      float " + ", ".join(cur) + ";")
        tdecl = [f"tx{l}_{i}" for l in need_l1 for i in range(0, 2 * l, 2)]
        if tdecl:
            L.append("      eelg_f2r " + ", ".join(tdecl) + ";")
        need_y0 = sorted({l * l + j for l in need_l2 for j in range(2 * l + 1)})
        L.append("      eelg_f4r " + ", ".join(f"ty{blk}" for blk in sorted({j // 4 for j in need_y0})) + ";")
        # asm outputs are taken as ready when the statement ends: every destination register
        # (vector temporaries included) is threaded through the lgkmcnt wait before any use
        live, after = [], []
        for l in need_l1:
            d = 2 * l + 1
            L.append(f"      {{ const unsigned xa = imb + 4 * ({fo_x[l]} + u * {d});")
            i = 0
            while i < d:
                if i + 1 < d:
                    L.append(f"        asm volatile(\"ds_read2_b32 %0, %1 offset0:{i} offset1:{i + 1}\" : \"=v\"(tx{l}_{i}) : \"v\"(xa));")
                    live.append(f"tx{l}_{i}")
                    after.append(f"x{l}_{i} = tx{l}_{i}[0]; x{l}_{i + 1} = tx{l}_{i}[1];")
                    i += 2
                else:
                    L.append(f"        asm volatile(\"ds_read_b32 %0, %1 offset:{4 * i}\" : \"=v\"(x{l}_{i}) : \"v\"(xa));")
                    live.append(f"x{l}_{i}")
                    i += 1
            L.append("      }")
        need_y = sorted({l * l + j for l in need_l2 for j in range(2 * l + 1)})
        for blk in sorted({j // 4 for j in need_y}):
            L.append(f"      asm volatile(\"ds_read_b128 %0, %1 offset:{4 * fo_sh + 16 * blk}\" : \"=v\"(ty{blk}) : \"v\"(imb));")
            live.append(f"ty{blk}")
            after.append(" ".join(f"y{j} = ty{blk}[{j - 4 * blk}];" for j in need_y if j // 4 == blk))
        if bf:
            # bf16 weights: ds_read_u16, widened exactly after the wait
            L.append("      unsigned " + ", ".join(f"wr{p.slot}" for p in grp) + ";")
            L.append("      { const unsigned wa = imb + 2 * u;")
            for p in grp:
                L.append(f"        asm volatile(\"ds_read_u16 %0, %1 offset:{4 * fo_w[p.slot]}\" : \"=v\"(wr{p.slot}) : \"v\"(wa));")
                live.append(f"wr{p.slot}")
                after.append(f"w{p.slot} = __uint_as_float(wr{p.slot} << 16);")
            L.append("      }")
        else:
            L.append("      { const unsigned wa = imb + 4 * u;")
            for p in grp:
                L.append(f"        asm volatile(\"ds_read_b32 %0, %1 offset:{4 * fo_w[p.slot]}\" : \"=v\"(w{p.slot}) : \"v\"(wa));")
                live.append(f"w{p.slot}")
            L.append("      }")
        for k in range(0, len(live), 24):
            ops = ", ".join(f'"+v"({v})' for v in live[k: k + 24])
            L.append(f'      asm volatile("s_waitcnt lgkmcnt(0)" : {ops} : : "memory");')
        L += ["      " + a_ for a_ in after]
        L.append('      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read before the image is refilled')
        for h in (0, 1):
            L.append(f"      while (node_{h} < n1_{h} && nend_{h} == e_{h}) {{   // uniform")
            nost = " && inv_norm < -1.0e30f" if TP_FWD_NOSTORE else ""   # measurement variant only
            L.append(f"        if (hf == {h}{f' && u < {LW}' if LW < 32 else ''}{nost}) {{")
            L.append(f"          float* __restrict__ o = agg + (size_t)node_{h} * {dmid};")
            for p in grp:
                d3 = 2 * p.l3 + 1
                L.extend("          " + ln for ln in vec_store([f"a{p.slot}_{k}" for k in range(d3)], "o",
                                                             f"{p.out_off + cg * LW * d3} + u * {d3}", nt=bool(TP_FWD_ANT)))
            L.append("          " + " ".join(f"{a} = 0.0f;" for a in accs))
            L.append("        }")
            L.append(f"        ++node_{h}; nend_{h} = nend2_{h}; nend2_{h} = rowptr[min(node_{h} + 2, n1_{h})];")
            L.append("      }")
        L.append("      if (e_0 >= eend_0 && e_1 >= eend_1) break;")
        L += ["  " + ln for ln in issue("b", NBUF)]
        L += _glds_compute(grp, cur, accs)
        L.append("      ++e_0; ++e_1; " + ("b ^= 1;" if NBUF == 2 else f"b = b == {NBUF - 1} ? 0 : b + 1;"))
        L.append("    }")
        L.append('    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the wave')
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    return L


def bwf_slot_table(paths, target: Irreps) -> Dict[int, Tuple[int, float, int]]:
    """slot -> (weight offset of its 32 x 32 block, alpha, gy offset) in the output linear
    ``o3.Linear(irreps_mid.simplify(), target)``: irreps_mid is sorted by l3, so the slots of
    one l3 form one merged input block (mul 32 x their count), whose instruction's weight is
    [32·cnt, 32] row-major with alpha 1/sqrt(32·cnt); instructions run in l3 order.  The host
    checks this table against the Linear it is handed (``eelg_tp_bwf_slot``)."""
    cnt: Dict[int, int] = {}
    for p in paths:
        cnt[p.l3] = cnt.get(p.l3, 0) + 1
    woff, o = {}, 0
    for l3 in sorted(cnt):
        woff[l3] = o
        o += 32 * cnt[l3] * MUL
    tgt_off = {ir.l: off for (m, ir), off in zip(target, target.offsets())}
    seen: Dict[int, int] = {}
    tab = {}
    for p in sorted(paths, key=lambda p: p.slot):
        q = seen.get(p.l3, 0)
        seen[p.l3] = q + 1
        tab[p.slot] = (woff[p.l3] + q * 32 * MUL, 1.0 / math.sqrt(32 * cnt[p.l3]), tgt_off[p.l3])
    return tab


def _emit_tp_bwf(name, sfx, bgroups, paths, target, din, nshp, wn, node_off, bf, ld_w, st_w):
    """Fused backward of ``linear(tp_interaction(x, sh, w))`` w.r.t. x and w, from the linear's
    output gradient gy [N, target.dim] (mul 32).  A workgroup owns R receivers and one input
    block l1 (grid: tiles x groups, the groups of a tile on one XCD):
      1. grad_agg of the group's slots for the R receivers, G[r][s][u][m] =
         alpha(l3) Σ_j W_s[u][j] gy[r][off(l3) + j·d3 + m], on v_mfma_f32_32x32x2f32 (rows u,
         columns (r, m), K = j) into LDS -- the [N, dmid] grad_agg tensor of the unfused path
         (written by the linear's grad-x, read back by tp_bwd) never reaches HBM;
      2. each half-wave streams the in-edges of one receiver (receiver-sorted order: one
         contiguous range) with tp_bwd's per-path arithmetic, its grad_agg slices read from LDS,
         storing grad_w and the per-edge grad_x rows (gxe) as tp_bwd does."""
    WT = "unsigned short" if bf else "float"
    R = TP_BWF_R
    tab = bwf_slot_table(paths, target)
    tdim = target.dim
    L: List[str] = []
    tasks, tb, sgs, lds_of = [], [0], [], {}
    for grp in bgroups:
        off = 0
        for p in grp:
            d3 = 2 * p.l3 + 1
            lds_of[p.slot] = off
            wo, al, go = tab[p.slot]
            for ct in range((R * d3 + 31) // 32):
                tasks.append((d3, ct, off, wo, go, al))
            off += 32 * d3
        sgs.append(off)
        tb.append(len(tasks))
    sgmax = max(sgs)
    nbg = len(bgroups)
    tn = f"bwf_tasks_{name}"
    if not bf:   # one task table per structure (shared by the bf16-storage kernel)
        L.append(f"static __constant__ eelg_bwf_task {tn}[{len(tasks)}] = {{")
        L += [f"  {{{d3}, {ct}, {off}, {wo}, {go}, {flit(al)}}}," for d3, ct, off, wo, go, al in tasks]
        L.append("};")
        L.append(f"static __constant__ int bwf_tb_{name}[{nbg + 1}] = {{{', '.join(map(str, tb))}}};")
        L.append(f"static __constant__ int bwf_sg_{name}[{nbg}] = {{{', '.join(map(str, sgs))}}};")
        L.append(f"static const int bwf_slots_{name}[{len(paths)}][2] = {{"
                 + ", ".join(f"{{{tab[s][0]}, {tab[s][2]}}}" for s in sorted(tab)) + "};")
        L.append(f"static const float bwf_alpha_{name}[{len(paths)}] = {{"
                 + ", ".join(flit(tab[s][1]) for s in sorted(tab)) + "};")
    EM, NX, P1 = TP_BWF_EM, TP_BWF_NX, TP_BWF_P1PF
    L.append(f"__global__ __launch_bounds__(256) void tp_bwf_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ receiver,")
    L.append("    const int* __restrict__ rowptr, int n_nodes,")
    L.append("    const float* __restrict__ gy, const float* __restrict__ wl, float inv_norm,")
    L.append(f"    {WT}* __restrict__ gw, {WT}* __restrict__ gxe) {{")
    L.append(f"  __shared__ float Gs[{R * sgmax}];")
    L.append("  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, u = lane & 31, hf = lane >> 5;")
    # 1-D grid of 8 * nt8 * NBG blocks (eelg_capi.hip): block b runs on XCD b % 8; the NBG group
    # blocks of a tile are 8 apart (same XCD, dispatched together: gy rows and edge indices
    # shared through one L2)
    L.append(f"  const int bi = blockIdx.x >> 3, by = bi % {nbg};")
    L.append(f"  const int n0 = ((bi / {nbg}) * 8 + (blockIdx.x & 7)) * {R};")
    L.append("  if (n0 >= n_nodes) return;")
    L.append(f"  const int sg = bwf_sg_{name}[by];")
    # ---- stage 1: grad_agg of the group's slots for the tile (MFMA into LDS) ----
    # the operands of task t + 4 are loaded while task t's MFMAs run (P1)
    L.append(f"  const int t1 = bwf_tb_{name}[by + 1]{' * 0' if TP_BWF_SKIP == 2 else ''};")
    L.append("  int t = bwf_tb_" + name + "[by] + wave;")

    def p1_load(pre, tv):
        return [f"  eelg_bwf_task {pre}tk = {tn}[{tv} < t1 ? {tv} : t1 - 1];",
                f"  int {pre}col = {pre}tk.ct * 32 + u, {pre}r = {pre}col / {pre}tk.d3, {pre}m = {pre}col - {pre}r * {pre}tk.d3;",
                f"  bool {pre}ok = {tv} < t1 && {pre}r < {R} && n0 + {pre}r < n_nodes;",
                f"  eelg_f4a {pre}a0, {pre}a1, {pre}a2, {pre}a3; float {pre}b[16];",
                f"  {{ const float* __restrict__ gp = gy + (size_t)(n0 + ({pre}ok ? {pre}r : 0)) * {tdim} + {pre}tk.gyoff + {pre}m + hf * 16 * {pre}tk.d3;",
                f"    const eelg_f4a* __restrict__ wp = reinterpret_cast<const eelg_f4a*>(wl + {pre}tk.woff + u * 32 + hf * 16);",
                f"    {pre}a0 = wp[0]; {pre}a1 = wp[1]; {pre}a2 = wp[2]; {pre}a3 = wp[3];",
                "    " + " ".join(f"{pre}b[{st}] = {pre}ok ? gp[{st} * {pre}tk.d3] : 0.0f;" for st in range(16)) + " }"]
    if P1:
        L.append("  if (t < t1) {")
        L += ["  " + ln for ln in p1_load("", "t")]
        L.append("  for (;;) {")
        L += ["  " + ln for ln in p1_load("n", "t + 4")]
    else:
        L.append("  for (; t < t1; t += 4) {")
        L += p1_load("", "t")
    L.append("    eelg_f32x16v acc = {};")
    for st in range(16):
        L.append(f"    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a{st // 4}[{st % 4}], b[{st}], acc, 0, 0, 0);")
    L.append("    if (ok) {")
    L.append("      float* __restrict__ gd = Gs + r * sg + tk.lds + 4 * hf * tk.d3 + m;")
    L += ["      " + " ".join(f"gd[{(v & 3) + 8 * (v >> 2)} * tk.d3] = acc[{v}] * tk.alpha;" for v in range(v0, v0 + 4))
          for v0 in range(0, 16, 4)]
    L.append("    }")
    if P1:
        L.append("    t += 4;")
        L.append("    if (t >= t1) break;")
        L.append("    tk = ntk; col = ncol; r = nr; m = nm; ok = nok; a0 = na0; a1 = na1; a2 = na2; a3 = na3;")
        L.append("    " + " ".join(f"b[{st}] = nb[{st}];" for st in range(16)))
        L.append("  }}")
    else:
        L.append("  }")
    L.append("  __syncthreads();")
    # ---- stage 2: the tile's in-edges, tp_bwd's per-path arithmetic with grad_agg from LDS ----
    L.append("  const int hw = threadIdx.x >> 5;")
    if TP_BWF_SKIP == 1:
        L.append("  if (n_nodes > 0) return;")
    if EM:
        # edge-major: half-wave hw takes edges eb + hw, eb + hw + 8, ... of the tile's range
        L.append(f"  const int eb = rowptr[n0] + hw, ee = rowptr[min(n0 + {R}, n_nodes)];")
        ES = 8
    else:
        # receiver-major: half-wave hw streams the in-edges of receiver n0 + hw
        L.append(f"  if (hw >= {R} || n0 + hw >= n_nodes) return;")
        L.append("  const int eb = rowptr[n0 + hw], ee = rowptr[n0 + hw + 1];")
        ES = 1
    L.append("  if (eb >= ee) return;")
    L.append("  switch (by) {")
    PF = TP_BWD_PFD
    for gi, grp in enumerate(bgroups):
        l = grp[0].l1
        d = 2 * l + 1
        sg = sgs[gi]
        l2s = sorted({p.l2 for p in grp})
        xs_ = [f"x{l}_{i}" for i in range(d)]
        ys_ = [f"y{l2 * l2 + j}" for l2 in l2s for j in range(2 * l2 + 1)]
        p0 = grp[0]
        L.append(f"  case {gi}: {{ // input block l1 = {l}")
        if not EM:
            L.append(f"    const float* __restrict__ gr = Gs + hw * {sg};")

        def edge_loads(pref, sv, ev):
            out = [f"    {{ const float* __restrict__ xs = x + (size_t){sv} * {din};",
                   f"      const float* __restrict__ ye = sh + (size_t){ev} * {nshp};",
                   f"      const {WT}* __restrict__ we = w + (size_t){ev} * {wn} + u;"]
            out += ["      " + ln for ln in vec_load([pref + v for v in xs_], "xs", f"{node_off[l]} + u * {d}")]
            out += ["      " + ln for ln in sh_load(l2s, pref, "ye")]
            out.append(f"      {pref}w{p0.slot} = {ld_w(f'we[{p0.slot * MUL}]')};")
            out.append("    }")
            return out
        carried = xs_ + ys_ + [f"w{p0.slot}"]
        if NX:
            L.append("    float " + ", ".join(carried) + ";")
            L += edge_loads("", "sender[eb]", "eb")
        L.append(f"    for (int e = eb; e < ee; e += {ES}) {{")
        if NX:
            L.append(f"      const bool more = e + {ES} < ee;")
            L.append(f"      const int sn = more ? sender[e + {ES}] : 0, en = more ? e + {ES} : e;")
        else:
            L.append("      float " + ", ".join(carried) + ";")
            L += ["  " + ln for ln in edge_loads("", "sender[e]", "e")]
        if EM:
            L.append(f"      const float* __restrict__ gr = Gs + (receiver[e] - n0) * {sg};")
        L.append(f"      const {WT}* __restrict__ we = w + (size_t)e * {wn} + u;")
        L.append(f"      {WT}* __restrict__ gwe = gw + (size_t)e * {wn} + u;")
        L.append(f"      {WT}* __restrict__ gxo = gxe + (size_t)e * {din};")
        for i in range(d):
            L.append(f"      float gx{l}_{i} = 0.0f;")
        if NX:
            L.append("      float " + ", ".join("n" + v for v in carried) + ";")
        base_pin = xs_ + [f"gx{l}_{i}" for i in range(d)] + ys_
        wregs = {0: [f"w{p0.slot}"]}
        for pj in range(1, min(PF, len(grp))):
            L.append(f"      float w{grp[pj].slot} = {ld_w(f'we[{grp[pj].slot * MUL}]')};")
            wregs[pj] = [f"w{grp[pj].slot}"]
        for pi, p in enumerate(grp):
            d3 = 2 * p.l3 + 1
            d1 = 2 * p.l1 + 1
            if pi + PF < len(grp):
                q = grp[pi + PF]
                L.append(f"      float w{q.slot} = {ld_w(f'we[{q.slot * MUL}]')};")
                wregs[pi + PF] = [f"w{q.slot}"]
            if pi + 1 < len(grp):
                nxt_regs = wregs[pi + 1]
            elif NX:                         # next edge's loads in flight during the last path
                L += ["  " + ln for ln in edge_loads("n", "sn", "en")]
                nxt_regs = ["n" + v for v in carried]
            else:
                nxt_regs = []
            L.append(f"      {{ // slot {p.slot}: {p.l1} x {p.l2} -> {p.l3}")
            L.append(f"        const float* __restrict__ gs = gr + {lds_of[p.slot]} + u * {d3};")
            L.append("        const float " + ", ".join(f"g{p.slot}_{k} = gs[{k}]" for k in range(d3)) + ";")
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
            if TP_BWD_NT and not bf:
                L.append(f"        __builtin_nontemporal_store(cp * ({gexpr}), &gwe[{p.slot * MUL}]);")
            else:
                L.append(f"        gwe[{p.slot * MUL}] = {st_w(f'cp * ({gexpr})')};")
            L.append(f"        const float hw_ = cp * w{p.slot};")
            for i in range(d1):
                ts = [f"m{i}_{k} * g{p.slot}_{k}" for k in range(d3) if (i, k) in byik]
                if ts:
                    L.append(f"        gx{p.l1}_{i} = fmaf(hw_, {' + '.join(ts)}, gx{p.l1}_{i});")
            L.append("      }")
            L.append("      " + pin(base_pin + nxt_regs))
        if bf:
            L += [f"      gxo[{node_off[l]} + u * {d} + {i}] = eelg_f2bf(gx{l}_{i});" for i in range(d)]
        else:
            L += ["      " + ln for ln in vec_store([f"gx{l}_{i}" for i in range(d)], "gxo", f"{node_off[l]} + u * {d}",
                                                       nt=bool(TP_BWD_NT))]
        if NX:
            L.append("      " + " ".join(f"{v} = n{v};" for v in carried))
        L.append("    }")
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    return L


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
    groups = _group_paths(sorted(paths, key=lambda p: (p.l1, p.l2, p.l3)), TP_MAXACC_BF if bf else TP_MAXACC)
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
    L += _emit_tp_fwd_glds2(name, groups, din, nshp, dmid, wn, node_off, bf)

    # channel groups (mul = 64: two 32-channel groups on blockIdx.y; mul = 16: lanes 16..31 idle)
    CG, LW = _chan_groups()
    UC = "u" if (CG, LW) == (1, 32) else "uc"     # this lane's channel in the row layouts
    YSW = "blockIdx.y" if CG == 1 else f"blockIdx.y / {CG}"
    chan_head = ["  const int u = lane & 31;"]
    if CG > 1:
        chan_head.append(f"  const int uc = u + (blockIdx.y % {CG}) * 32;")
    elif LW < 32:
        chan_head += [f"  if (u >= {LW}) return;   // no channel", "  const int uc = u;"]
    # ---------------- backward (per edge) ----------------
    # grouped by input block l1: each group owns a disjoint slice of gxe, so no
    # cross-group reduction is needed; grad_w of every path is written once.
    bgroups = [[p for p in paths if p.l1 == l] for l in node_ls]
    bgroups = [g for g in bgroups if g]
    NBG = len(bgroups) * CG
    bwpe = f" __attribute__((amdgpu_waves_per_eu({TP_BWD_WPE})))" if TP_BWD_WPE else ""
    L.append(f"__global__ __launch_bounds__(256){bwpe} void tp_bwd_{name}{sfx}(")
    L.append(f"    const float* __restrict__ x, const float* __restrict__ sh, const {WT}* __restrict__ w,")
    L.append("    const int* __restrict__ sender, const int* __restrict__ receiver, int n_edges,")
    L.append("    const float* __restrict__ gagg, float inv_norm,")
    L.append(f"    {WT}* __restrict__ gw, {WT}* __restrict__ gxe, const int* __restrict__ spos) {{")
    L.append("  const int lane = threadIdx.x & 63;")
    if TP_BWD_XCD:
        # 1-D grid of 8 * nb8 * NBG blocks (eelg_capi.hip); block b runs on XCD b % 8, which
        # takes edge blocks [xcd * nb8, (xcd + 1) * nb8); surplus edge blocks exit below
        L.append(f"  const int nb8 = gridDim.x / {8 * NBG}, xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;")
        if TP_BWD_XCD == 1:
            L.append(f"  const int by = bi % {NBG}, bx = xcd * nb8 + bi / {NBG};")
        else:
            L.append(f"  const int by = bi / nb8, bx = xcd * nb8 + bi % nb8;")
    else:
        L.append("  const int by = blockIdx.y, bx = blockIdx.x;")
    L += [ln.replace("blockIdx.y", "by") for ln in chan_head]
    # spos (optional): gxe row of edge e is spos[e], its position in sender order, so the sender
    # sum reads gxe contiguously instead of gathering rows through sperm
    # a half-wave streams TP_BWD_EPH consecutive edges: while the last path of edge e
    # computes, edge e+1's x / SH rows and first path's grad_agg slice and weight are in
    # flight (its sender / receiver indices were loaded when edge e started)
    EPH = TP_BWD_EPH
    L.append(f"  const int e0 = ((bx * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5)) * {EPH};")
    L.append("  if (e0 >= n_edges) return;")
    L.append(f"  const int e1 = min(e0 + {EPH}, n_edges);")
    L.append(f"  switch ({YSW.replace('blockIdx.y', 'by')}) {{")
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
                   f"      const {WT}* __restrict__ we = w + (size_t){ev} * {wn} + {UC};"]
            out += ["      " + ln for ln in vec_load([pref + v for v in xs_], "xs", f"{node_off[l]} + {UC} * {d}")]
            out += ["      " + ln for ln in sh_load(l2s, pref, "ye")]
            d3 = 2 * p0.l3 + 1
            out += ["      " + ln for ln in vec_load([f"{pref}g{p0.slot}_{k}" for k in range(d3)], "ge",
                                                      f"{p0.out_off} + {UC} * {d3}")]
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
        L.append(f"      const {WT}* __restrict__ we = w + (size_t)e * {wn} + {UC};")
        L.append(f"      {WT}* __restrict__ gwe = gw + (size_t)e * {wn} + {UC};")
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
                                                    f"{p.out_off} + {UC} * {d3}")]
            out.append(f"      float w{p.slot} = {ld_w(f'we[{p.slot * MUL}]')};")
            return out, [f"g{p.slot}_{k}" for k in range(d3)] + [f"w{p.slot}"]
        PF = TP_BWD_PFD
        regs_of = {}
        for pj in range(1, min(PF, len(grp))):   # paths 1 .. PF-1 issued up front
            code, regs_of[pj] = pref(grp[pj])
            L += code
        for pi, p in enumerate(grp):
            d3 = 2 * p.l3 + 1
            d1 = 2 * p.l1 + 1
            if pi + PF < len(grp):           # path pi + PF's loads in flight during this one
                code, regs_of[pi + PF] = pref(grp[pi + PF])
                L += code
            if pi + 1 < len(grp):
                # only the next path must have landed after this one; later paths stay in flight
                nxt_regs = regs_of[pi + 1]
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
            if TP_BWD_NT and not bf:
                L.append(f"        __builtin_nontemporal_store(cp * ({gexpr}), &gwe[{p.slot * MUL}]);")
            else:
                L.append(f"        gwe[{p.slot * MUL}] = {st_w(f'cp * ({gexpr})')};")
            L.append(f"        const float hw = cp * w{p.slot};")
            for i in range(d1):
                ts = [f"m{i}_{k} * g{p.slot}_{k}" for k in range(d3) if (i, k) in byik]
                if ts:
                    L.append(f"        gx{p.l1}_{i} = fmaf(hw, {' + '.join(ts)}, gx{p.l1}_{i});")
            L.append("      }")
            L.append("      " + pin(base_pin + nxt_regs))
        if bf:
            L += [f"      gxo[{node_off[l]} + {UC} * {d} + {i}] = eelg_f2bf(gx{l}_{i});" for i in range(d)]
        else:
            L += ["      " + ln for ln in vec_store([f"gx{l}_{i}" for i in range(d)], "gxo", f"{node_off[l]} + {UC} * {d}",
                                                       nt=bool(TP_BWD_NT))]
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
    L += chan_head
    L.append("  const int n = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);")
    L.append("  if (n >= n_nodes) return;")
    L.append("  const int p0 = srowptr[n], p1 = srowptr[n + 1];")
    L.append(f"  switch ({YSW}) {{")
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
        L += ["      " + ln for ln in vec_load(xs_, "xs", f"{node_off[l]} + {UC} * {d}")]
        L.append("    }")
        L.append("    float " + ", ".join(f"{v} = 0.0f" for v in gxs) + ";")
        L.append("    int en = p0 < p1 ? sperm[p0] : 0;")
        L.append("    for (int p = p0; p < p1; ++p) {")
        L.append("      const int e = en;")
        L.append("      en = p + 1 < p1 ? sperm[p + 1] : 0;")
        L.append("      const int r = receiver[e];")
        L.append(f"      const float* __restrict__ ye = sh + (size_t)e * {nshp};")
        L.append(f"      const float* __restrict__ ge = gagg + (size_t)r * {dmid};")
        L.append(f"      const {WT}* __restrict__ we = w + (size_t)e * {wn} + {UC};")
        L.append(f"      {WT}* __restrict__ gwe = gw + (size_t)e * {wn} + {UC};")
        L.append("      float " + ", ".join(ys_) + ";")
        L += ["      " + ln for ln in sh_load(l2s, "", "ye")]

        def pload(p):
            d3 = 2 * p.l3 + 1
            out = ["      float " + ", ".join(f"g{p.slot}_{k}" for k in range(d3)) + ";"]
            out += ["      " + ln for ln in vec_load([f"g{p.slot}_{k}" for k in range(d3)], "ge",
                                                    f"{p.out_off} + {UC} * {d3}")]
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
        L += ["    " + ln for ln in vec_store(gxs, "gxo", f"{node_off[l]} + {UC} * {d}")]
        L.append("    break; }")
    L.append("  default: break;")
    L.append("  }")
    L.append("}")
    # fused output-linear grad-x + backward (mul 32: one channel group of 32 lanes)
    bwf = CG == 1 and LW == 32
    if bwf:
        L += _emit_tp_bwf(name, sfx, bgroups, paths, target, din, nshp, wn, node_off, bf, ld_w, st_w)
    info = dict(din=din, dmid=dmid, wn=wn, nsh=nsh, ngroups=len(groups) * CG, nbgroups=len(bgroups) * CG,
                npaths=len(paths), nph=TP_NPH, beph=TP_BWD_EPH, fwpb=TP_FWD_WPB, bxcd=TP_BWD_XCD,
                bwf=int(bwf), bwf_r=TP_BWF_R, tdim=target.dim,
                sig=fnv1a64(tp_signature(node, sh, target)))
    return "\n".join(L), info


# ---------------------------------------------------------------------------
# symmetric contraction
# ---------------------------------------------------------------------------
def pin(vs: List[str], memory: bool = False, sgprs: Sequence[str] = ()) -> str:
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
    """Pack the polynomial terms into blocks of <= maxb terms, in term order.  A block holds
    the deg-1 terms or a run of (a, b) pair segments: several whole pairs, or part of one (a
    pair is split only at c-subgroup boundaries, and a c-subgroup longer than maxb stays whole).
    Each block's coefficients are prefetched into SGPRs while earlier blocks compute, so blocks
    of similar size keep that prefetch distance even where the pairs are small."""
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
    cur = None

    def new_block():
        blk = {"kind": "pairs", "segs": [], "terms": []}
        blocks.append(blk)
        return blk
    for (a, b), g in pairs.items():
        units = ([("d2", g["d2"])] if g["d2"] else []) + [(c, lst) for c, lst in g["d3"].items()]
        seg = None
        for kind, lst in units:
            if cur is None or (cur["terms"] and len(cur["terms"]) + len(lst) > maxb):
                if seg is not None:
                    seg["last"] = False
                cur = new_block()
                seg = None
            if seg is None:
                seg = {"a": a, "b": b, "first": not any(s_["a"] == a and s_["b"] == b
                                                        for b_ in blocks for s_ in b_.get("segs", [])),
                       "last": True, "d2": [], "d3": []}
                cur["segs"].append(seg)
            if kind == "d2":
                seg["d2"] += lst
            else:
                seg["d3"].append((kind, lst))
            cur["terms"] += [t for t, _ in lst]
    return blocks


def _coef_cost(plan, g) -> int:
    """issue cost of one term group per node: 4 x its operands (the LDS reads, round-2 model)
    or its VALU count (one FMA per term + the shared pair / triple products), the larger"""
    ops, prods = set(), set()
    for t in g:
        nu, (a, b, c), q = plan.terms[t]
        ops |= {("x", a), ("g", q)} | ({("x", b)} if nu >= 2 else set()) | ({("x", c)} if nu >= 3 else set())
        prods |= ({(a, b)} if nu >= 2 else set()) | ({(a, b, c)} if nu >= 3 else set())
    return max(4 * len(ops), len(prods) + len(g))


def coef_sets(plan, n_sets: int, n_waves: int, jg: int) -> List[List[int]]:
    """Term groups of the streaming coefficient gradient: ``n_sets * n_waves`` clustered groups
    (``coef_groups``), one per wave, returned in launch order (group s * n_waves + w = set s,
    wave w).  Every chunk ends in a workgroup barrier, so a step lasts as long as the busiest
    SIMD's waves; waves w, w + 4, w + 8, w + 12 share a SIMD (cyclic wave placement), so the
    groups are dealt longest-first to the (set, w mod 4) bin with the least work."""
    groups = [g for g in coef_groups(plan, 1, jg, n_sets * n_waves, pairs=bool(SC_COEF_PAIRS)) if g]
    assert len(groups) <= n_sets * n_waves, (len(groups), n_sets, n_waves)
    per = n_waves // 4
    bins = {(st, k): [] for st in range(n_sets) for k in range(4)}
    load = {b: 0 for b in bins}
    for g in sorted(groups, key=lambda g: _coef_cost(plan, g), reverse=True):
        b = min((b for b in bins if len(bins[b]) < per), key=lambda b: load[b])
        bins[b].append(g)
        load[b] += _coef_cost(plan, g)
    out = []
    for st in range(n_sets):
        for w in range(n_waves):
            lst = bins[(st, w % 4)]
            out.append(lst[w // 4] if w // 4 < len(lst) else [])
    return out


def coef_groups(plan, n_waves: int, jg: int, n_groups: int, lds_w: int = 2,
                pairs: bool = False) -> List[List[int]]:
    """Term groups of the coefficient gradient, clustered so that a group reads few operands.

    A lane (one node) of a group loads every x_a / g_q the group's terms use from LDS once per
    64-node sub-tile, and the LDS operand reads, not the VALU, bounded the kernel when groups
    were runs of the term order (35 operands per 59 terms: 16 waves x 35 x 2 LDS cycles per CU
    against 4 waves x 85 x 2 VALU cycles per SIMD).  Greedy clustering: a group grows by the
    term adding the fewest ``lds_w`` x new operands + new products (x_a x_b, x_a x_b x_c), so
    the operand union drops to ~18 and the VALU count (one FMA per term + the shared products)
    becomes the bound.  The groups are then dealt to the waves longest-first (each wave takes
    n_groups / n_waves of them; a workgroup holds its CU until its slowest wave ends), and
    returned in launch order: group k * n_waves + w belongs to wave w."""
    import numpy as np
    terms = plan.terms
    nt = len(terms)
    opm = np.zeros(nt, dtype=np.uint64)
    abid = np.full(nt, -1, dtype=np.int64)
    abcid = np.full(nt, -1, dtype=np.int64)
    ab_ix, abc_ix = {}, {}
    nx = 1 + max(max(a, b, c) for _, (a, b, c), _ in terms)
    # pairs: an operand costs its LDS row pair (rows 2p, 2p + 1: one ds_read_b64 of the
    # streaming kernel's image), so the groups gather operands whose partner row is used too
    f = (lambda i: i // 2) if pairs else (lambda i: i)  # noqa: E731
    for t, (nu, (a, b, c), q) in enumerate(terms):
        m = (1 << f(a)) | (1 << (nx + f(q)))
        if nu >= 2:
            m |= 1 << f(b)
            abid[t] = ab_ix.setdefault((a, b), len(ab_ix))
        if nu >= 3:
            m |= 1 << f(c)
            abcid[t] = abc_ix.setdefault((a, b, c), len(abc_ix))
        opm[t] = m
    assert 2 * nx <= 64
    left = np.ones(nt, dtype=bool)
    groups = []
    BIG = np.int64(1 << 40)
    while left.any():
        g = [int(np.argmax(left))]
        left[g[0]] = False
        um = opm[g[0]]
        hab = np.zeros(len(ab_ix) + 1, dtype=bool)
        habc = np.zeros(len(abc_ix) + 1, dtype=bool)
        hab[abid[g[0]]] = True
        habc[abcid[g[0]]] = True
        while len(g) < jg and left.any():
            new_ops = np.bitwise_count(opm & ~um).astype(np.int64)
            cost = (lds_w * new_ops + (~hab[abid] & (abid >= 0)) + (~habc[abcid] & (abcid >= 0)))
            cost = np.where(left, cost, BIG)
            t = int(np.argmin(cost))
            g.append(t)
            left[t] = False
            um |= opm[t]
            hab[abid[t]] = True
            habc[abcid[t]] = True
        groups.append(g)
    assert len(groups) <= n_groups, (len(groups), n_groups)

    def cost(g):
        return _coef_cost(plan, g)
    per = n_groups // n_waves
    load = [0] * n_waves
    slots: List[List[List[int]]] = [[] for _ in range(n_waves)]
    for g in sorted(groups, key=cost, reverse=True):
        w = min((w for w in range(n_waves) if len(slots[w]) < per), key=lambda w: load[w])
        slots[w].append(g)
        load[w] += cost(g)
    out = []
    for k in range(per):
        for w in range(n_waves):
            out.append(slots[w][k] if k < len(slots[w]) else [])
    return out


def _pk_cload(blk, CE):
    if SC_PK_MODE == "dual":
        return _pk_cload_dual(blk, CE)
    if SC_PK_MODE == "pairs":
        return _pk_cload_pairs(blk, CE)
    return _pk_cload_asm(blk, CE)


def _pk_cload_pairs(blk, CE):
    """One 8-byte scalar load per coefficient, at its own offset: the coefficient is the low
    half of its own aligned SGPR pair (the compiler merges neighbouring loads into wider ones)
    and only pairs are pinned, never whole vectors"""
    ts = blk["terms"]
    out, names = [], []
    for t in ts:
        nm = f"cp{t}"
        out.append(f"  eelg_c2 {nm} = *reinterpret_cast<const eelg_c2*>(cf + {t});")
        CE[t] = (f"eelg_splat({nm}, 0)", 0)
        names.append(nm)
    return out, names


def _pk_cload_dual(blk, CE):
    """Two scalar-load sets of a block's coefficients, at t0 and at t0 + 1 (16 / 8 / 4 / 2 terms
    per load; rows are padded past the last term): term t0 + i is element i of the first set for
    even i and element i - 1 of the second for odd i, always an even element, i.e. the low half
    of an aligned SGPR pair.  CE[t] = the splat expression."""
    ts = blk["terms"]
    t0, n = ts[0], len(ts)
    assert ts == list(range(t0, t0 + n))
    out, names = [], []
    for sh, tag in ((0, "a"), (1, "b")):
        t = t0 + sh
        cnt = n - sh
        while cnt > 0:
            sz = next(z for z in (16, 8, 4, 2) if z <= max(cnt, 2))
            nm = f"cv{tag}{t}"
            out.append(f"  eelg_c{sz} {nm} = *reinterpret_cast<const eelg_c{sz}*>(cf + {t});")
            for i in range(0, min(sz, cnt), 2):
                CE[t + i] = (f"eelg_splat({nm}, {i})", 0)
            names.append(nm)
            t += sz
            cnt -= sz
    return out, names


def _pk_cload_asm(blk, CE):
    """Scalar loads of a block's coefficients as SGPR vectors of 16 / 8 / 4 / 2 terms (an odd tail
    is loaded as a pair: the row is padded past the last term).  CE[t] = (pair expression, half):
    the aligned SGPR pair holding coefficient t, and which half of it (op_sel)."""
    ts = blk["terms"]
    t0, n = ts[0], len(ts)
    assert ts == list(range(t0, t0 + n))
    out, names, t = [], [], t0
    while t < t0 + n:
        left = t0 + n - t
        sz = next(z for z in (16, 8, 4, 2) if z <= max(left, 2))
        nm = f"cv{t}"
        out.append(f"  eelg_c{sz} {nm} = *reinterpret_cast<const eelg_c{sz}*>(cf + {t});")
        for i in range(min(sz, left)):
            CE[t + i] = (f"eelg_pair({nm}, {i // 2})" if sz > 2 else nm, i % 2)
        names.append(nm)
        t += sz
    return out, names


class _PkSched:
    """The packed VALU stream of one coefficient block as a list of instructions (macro text,
    written variables, read variables), emitted as ``asm volatile`` in a dependency-respecting
    order that keeps every consumer at least one instruction behind its producer.  The hazard
    recognizer puts an ``s_nop`` before an inline-asm reader of a VGPR that one of the two
    preceding VALU instructions wrote (2857 / 5801 of them in sc_fwd / sc_bwd_x of sc_l4_c3
    before this order),
    and the compiler's scheduler places products right before their first use; a fixed order of
    volatile statements leaves it nothing to undo.  A small look-ahead window bounds the register
    live ranges."""

    def __init__(self, window=10, dist=2):
        self.ins = []
        self.window = window
        self.dist = dist            # keep a reader at least this many instructions behind

    def add(self, text, writes, reads):
        self.ins.append((text, tuple(writes), tuple(reads)))

    def emit(self, ind="  "):
        n = len(self.ins)
        if not SC_PK_SCHED:
            out = [ind + t for t, _, _ in self.ins]
            self.ins = []
            return out
        deps = [set() for _ in range(n)]
        last_w, reads_since = {}, {}
        for j, (_, w, r) in enumerate(self.ins):
            for v in r:
                if v in last_w:
                    deps[j].add(last_w[v])              # RAW
            for v in w:
                if v in last_w:
                    deps[j].add(last_w[v])              # WAW
                for i in reads_since.get(v, ()):
                    if i != j:
                        deps[j].add(i)                  # WAR
            for v in r:
                reads_since.setdefault(v, []).append(j)
            for v in w:
                last_w[v] = j
                reads_since[v] = []
        done, out, recent = [False] * n, [], []
        pending = list(range(n))
        while pending:
            pick, best = None, None
            for j in pending[: self.window]:
                if all(done[i] for i in deps[j]):
                    # distance to the nearest recent producer of an operand (0 = none recent)
                    near = next((k for k, w in enumerate(reversed(recent), 1)
                                 if set(self.ins[j][2]) & set(w)), 0)
                    if near == 0:
                        pick = j
                        break
                    if best is None or near > best:
                        pick, best = j, near
            j = pick
            done[j] = True
            pending.remove(j)
            out.append(ind + self.ins[j][0])
            recent = (recent + [self.ins[j][1]])[-self.dist:]
        self.ins = []
        return out


def emit_sc_packed(L, name, plan, lin, lout, D, Dout, TP, NB, NTH, head, stage_in, stage_out,
                   cm_store, lq):
    """sc_fwd / sc_bwd_x with two nodes per lane (tile rows lane and lane + 64) on packed fp32:
    every coefficient FMA is one v_pk_fma_f32 whose SGPR operand broadcasts one half of an aligned
    coefficient pair (EELG_PKF_LO / _HI), the pair / triple products and the grad-x chain are
    v_pk_mul_f32 / v_pk_fma_f32 on VGPRs (EELG_PKMV / EELG_PKFV), all scheduled by _PkSched.
    Same blocks, prefetch and pins as the plain form."""
    CE = {}
    S = _PkSched()

    def cfma(t, b, c):
        pr, hf = CE[t]
        if SC_PK_MODE in ("dual", "pairs"):
            S.add(f"{c} = __builtin_elementwise_fma({pr}, {b}, {c});", [c], [c, b])
        else:
            S.add(f"EELG_PKF_{'HI' if hf else 'LO'}({c}, {pr}, {b});", [c], [c, b])

    def cmul(t, b, c):
        pr, hf = CE[t]
        if SC_PK_MODE in ("dual", "pairs"):
            S.add(f"{c} = __builtin_elementwise_fma({pr}, {b}, (eelg_f2r){{0.0f, 0.0f}});", [c], [b])
        else:
            S.add(f"EELG_PKM_{'HI' if hf else 'LO'}({c}, {pr}, {b});", [c], [b])

    def vmul(d, a, b):
        S.add(f"EELG_PKMV({d}, {a}, {b});", [d], [a, b])

    def vfma(d, a, b):
        S.add(f"EELG_PKFV({d}, {a}, {b});", [d], [d, a, b])

    rows = [f"  float* __restrict__ tr0 = tile + lane * {TP};",
            f"  float* __restrict__ tr1 = tile + (lane + 64) * {TP};"]

    def ld2(col):
        return f"(eelg_f2r){{tr0[{col}], tr1[{col}]}}"

    # ---------------- forward ----------------
    L.append(f"__global__ __launch_bounds__({NTH}) void sc_fwd_{name}(")
    L.append("    const float* __restrict__ x, const float* __restrict__ coef, int n_nodes,")
    L.append("    float* __restrict__ out) {")
    L.append(f"  __shared__ float tile[{NB} * {TP}];")
    L += head
    L += stage_in("x", "tile", lin, NB, NTH)
    L.append("  __syncthreads();")
    L += rows
    for a in range(D):
        L.append(f"  eelg_f2r x{a} = {ld2(lq(lin, a, 'cl'))};")
    blocks = sc_blocks(plan, SC_BLOCK_FWD)
    fv = [f"x{a}" for a in range(D)]
    pf = {}
    for j in range(min(SC_PFD_FWD, len(blocks))):
        lines, pf[j] = _pk_cload(blocks[j], CE)
        L += lines
    declared = set()
    for q in range(Dout):
        L.append(f"  eelg_f2r o{q};")

    def acc(t, q, b):
        # the first term into o_q is a multiply (no zero fill of the accumulators)
        if q in declared:
            cfma(t, b, f"o{q}")
        else:
            cmul(t, b, f"o{q}")
            declared.add(q)
    pdecl = set()
    for bi, blk in enumerate(blocks):
        if bi + SC_PFD_FWD < len(blocks):
            lines, pf[bi + SC_PFD_FWD] = _pk_cload(blocks[bi + SC_PFD_FWD], CE)
            L += lines
        nxt = [nm for j in range(bi + 1, bi + 1 + SC_PFD_FWD) for nm in pf.get(j, [])]
        carry = []
        tmp = []
        if blk["kind"] == "deg1":
            for t, a, q in blk["deg1"]:
                acc(t, q, f"x{a}")
        for sg in blk.get("segs", []):
            a, b = sg["a"], sg["b"]
            pv = f"p{a}_{b}"
            if sg["first"]:
                pdecl.add(pv)
                L.append(f"  eelg_f2r {pv};")
                vmul(pv, f"x{a}", f"x{b}")
            for t, q in sg["d2"]:
                acc(t, q, pv)
            for cc, lst in sg["d3"]:
                mv = f"m{a}_{b}_{cc}"
                tmp.append(mv)
                vmul(mv, pv, f"x{cc}")
                for t, q in lst:
                    acc(t, q, mv)
            if not sg["last"]:
                carry = [pv]
        if tmp:
            L.append("  eelg_f2r " + ", ".join(tmp) + ";")
        L.append("  {")
        L += S.emit("    ")
        L.append("  }")
        L.append("  " + pin(fv + sorted(f"o{q}" for q in declared) + carry, sgprs=nxt))
    for q in range(Dout):
        if q not in declared:
            L.append(f"  o{q} = (eelg_f2r){{0.0f, 0.0f}};")
    L.append("  __syncthreads();")
    for q in range(Dout):
        col = lq(lout, q, 'cl')
        L.append(f"  tr0[{col}] = o{q}.x; tr1[{col}] = o{q}.y;")
    L.append("  __syncthreads();")
    L += stage_out("out", "tile", lout, NB, NTH)
    L.append("}")

    # ---------------- backward w.r.t. x ----------------
    CE.clear()
    L.append(f"__global__ __launch_bounds__({NTH}) void sc_bwd_x_{name}(")
    L.append("    const float* __restrict__ x, const float* __restrict__ coef,")
    L.append("    const float* __restrict__ gout, int n_nodes, float* __restrict__ gx,")
    L.append("    float* __restrict__ xt, float* __restrict__ gt) {")
    L.append(f"  __shared__ float tile[{NB} * {TP}];")
    L += head
    L += stage_in("x", "tile", lin, NB, NTH)
    L.append("  __syncthreads();")
    L.append("  if (xt) {")
    L += cm_store("xt", "tile", lin, NB, "    ", NTH)
    L.append("  }")
    L += rows
    for a in range(D):
        L.append(f"  eelg_f2r x{a} = {ld2(lq(lin, a, 'cl'))};")
    L.append("  __syncthreads();")
    L += stage_in("gout", "tile", lout, NB, NTH)
    L.append("  __syncthreads();")
    L.append("  if (gt) {")
    L += cm_store("gt", "tile", lout, NB, "    ", NTH)
    L.append("  }")
    for q in range(Dout):
        L.append(f"  eelg_f2r g{q} = {ld2(lq(lout, q, 'cl'))};")
    dset = set()
    for a in range(D):
        L.append(f"  eelg_f2r d{a};")
    blocks = sc_blocks(plan, SC_PK_BLOCK_BWD)
    pf = {}
    for j in range(min(SC_PFD_BWD, len(blocks))):
        lines, pf[j] = _pk_cload(blocks[j], CE)
        L += lines

    def dacc(a, u, v):
        """d_a += u * v (the first contribution a multiply)"""
        if a in dset:
            vfma(f"d{a}", u, v)
        else:
            vmul(f"d{a}", u, v)
            dset.add(a)
    for bi, blk in enumerate(blocks):
        if bi + SC_PFD_BWD < len(blocks):
            lines, pf[bi + SC_PFD_BWD] = _pk_cload(blocks[bi + SC_PFD_BWD], CE)
            L += lines
        nxt = [nm for j in range(bi + 1, bi + 1 + SC_PFD_BWD) for nm in pf.get(j, [])]
        carry = []
        tmp = []
        if blk["kind"] == "deg1":
            for t, a, q in blk["deg1"]:
                if a in dset:
                    cfma(t, f"g{q}", f"d{a}")
                else:
                    cmul(t, f"g{q}", f"d{a}")
                    dset.add(a)
        for sg in blk.get("segs", []):
            a, b = sg["a"], sg["b"]
            pv, sv = f"p{a}_{b}", f"s{a}_{b}"
            first_sv = True
            if sg["first"]:
                L.append(f"  eelg_f2r {pv}, {sv};")
                vmul(pv, f"x{a}", f"x{b}")
            else:
                first_sv = False                      # carried in from the previous block
            for t, q in sg["d2"]:
                if first_sv:
                    cmul(t, f"g{q}", sv)
                    first_sv = False
                else:
                    cfma(t, f"g{q}", sv)
            for cc, lst in sg["d3"]:
                s = f"s{a}_{b}_{cc}"
                tmp.append(s)
                for k, (t, q) in enumerate(lst):
                    (cmul if k == 0 else cfma)(t, f"g{q}", s)
                dacc(cc, s, pv)
                if first_sv:
                    vmul(sv, s, f"x{cc}")
                    first_sv = False
                else:
                    vfma(sv, s, f"x{cc}")
            if sg["last"]:
                if first_sv:
                    raise AssertionError("a pair segment with no terms")
                dacc(a, sv, f"x{b}")
                dacc(b, sv, f"x{a}")
            else:
                carry = [pv, sv]
        if tmp:
            L.append("  eelg_f2r " + ", ".join(tmp) + ";")
        L.append("  {")
        L += S.emit("    ")
        L.append("  }")
        bv = ([f"x{a}" for a in range(D)] + [f"g{q}" for q in range(Dout)] +
              sorted(f"d{a}" for a in dset))
        L.append("  " + pin(bv + carry, sgprs=nxt))
    for a in range(D):
        if a not in dset:
            L.append(f"  d{a} = (eelg_f2r){{0.0f, 0.0f}};")
    L.append("  __syncthreads();")
    for a in range(D):
        col = lq(lin, a, 'cl')
        L.append(f"  tr0[{col}] = d{a}.x; tr1[{col}] = d{a}.y;")
    L.append("  __syncthreads();")
    L += stage_out("gx", "tile", lin, NB, NTH)
    L.append("}")


def emit_sc(name: str, coupling: str, ls: Tuple[int, ...], corr: int) -> Tuple[str, dict]:
    """Symmetric contraction kernels.

    Layout: x / out rows are e3nn mul-major ([l-block][channel][m]); a workgroup
    of 4 waves owns 4 consecutive channels ("channel quad") x 64 nodes and stages
    the quad's 4*D floats per node through LDS with contiguous global segments, so
    every byte of x / out crosses HBM once.  One wave = one channel (wave-uniform,
    coefficients come through scalar loads), one lane = one node.  The output irreps
    (``ls``, parity (-1)^l) may differ from the coupling irreps of the input (the
    reference's product block maps the interaction irreps onto the hidden irreps)."""
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
    # coefficient row stride: 64-B aligned channel rows, at least one float past the last term (the
    # packed kernels load coefficients in pairs)
    cld = -(-(nt + (1 if SC_PK else 0)) // 16) * 16

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

    NB = 128 if SC_PK else 64 * SC_NT        # nodes per workgroup (fwd / grad-x): one (two packed) per lane
    NTH = 256 * SC_NT                       # threads per workgroup (fwd / grad-x)
    VT = "float"

    def vfma(a, b, c):
        return f"fmaf({a}, {b}, {c})"

    def cfma(t, b, c):
        """c += coefficient t * b (the coefficient is a wave-uniform SGPR)"""
        return vfma(CE[t], b, c)
    CE: Dict[int, str] = {}                 # term -> expression of its (SGPR) coefficient

    def cload(blk):
        """the scalar loads of block blk's coefficients (a contiguous term range) and the names
        to pin; records every term's coefficient expression in CE"""
        ts = blk["terms"]
        t0, n = ts[0], len(ts)
        assert ts == list(range(t0, t0 + n))
        if not SC_CVEC:
            for t in ts:
                CE[t] = f"c{t}"
            return [f"  float c{t} = cf[{t}];" for t in ts], [f"c{t}" for t in ts]
        out, names, t = [], [], t0
        while t < t0 + n:
            sz = next(z for z in (16, 8, 4, 2, 1) if z <= t0 + n - t)
            nm = f"cv{t}"
            if sz == 1:
                out.append(f"  float {nm} = cf[{t}];")
                CE[t] = nm
            else:
                out.append(f"  eelg_c{sz} {nm} = *reinterpret_cast<const eelg_c{sz}*>(cf + {t});")
                for i in range(sz):
                    CE[t + i] = f"{nm}[{i}]"
            names.append(nm)
            t += sz
        return out, names
    zero = "0.0f"

    def lds_get(ptr, col):
        return f"{ptr}[{col}]"

    def lds_put(ptr, col, v):
        return f"{ptr}[{col}] = {v};"

    # Staging between the mul-major rows and the quad tile.  A quad owns, per node and l-block,
    # one run of 4*d floats (d float4, 16-B aligned), so a tile of nb nodes is nb * D float4:
    # float4 j of a node sits at LDS column 4*j and at global float offset
    # o_l + cq*4*d_l + 4*(j - start_l) of its l-block.  Every float4 load of a thread is issued
    # before the first LDS store (one memory round trip per tile, not one per element), with
    # the node index clamped in bounds instead of a branch around each load.
    def _gofs(lay, j):
        """select chain (v_cndmask, no branches): global float offset of quad float4 j"""
        expr = None
        for (s0, s1, o, d) in lay.segs:
            st4 = s0 // 4
            v = f"{o} + cqo_ * {4 * d} + 4 * ({j} - {st4})"
            expr = v if expr is None else f"({j} >= {st4} ? {v} : {expr})"
        return expr

    def stage_in(src, tile, lay, nb=64, nth=256):
        n4 = lay.QD // 4
        tot = nb * n4
        it_n = -(-tot // nth)
        out = ["  { int cqo_ = cq; asm volatile(\"\" : \"+s\"(cqo_));"]
        for it in range(it_n):
            out.append(f"    const int i{it} = min((int)threadIdx.x + {nth * it}, {tot - 1}), "
                       f"nl{it} = i{it} / {n4}, j{it} = i{it} - nl{it} * {n4};")
            out.append(f"    const float4 v{it} = *reinterpret_cast<const float4*>({src} + "
                       f"(size_t)min(n0 + nl{it}, n_nodes - 1) * {lay.row} + {_gofs(lay, f'j{it}')});")
        for it in range(it_n):
            # a clamped tail thread rewrites the tile's last float4 with the same value
            out.append(f"    {{ const bool ok = n0 + nl{it} < n_nodes; "
                       f"float* t_ = {tile} + nl{it} * {TP} + 4 * j{it}; "
                       f"t_[0] = ok ? v{it}.x : 0.0f; t_[1] = ok ? v{it}.y : 0.0f; "
                       f"t_[2] = ok ? v{it}.z : 0.0f; t_[3] = ok ? v{it}.w : 0.0f; }}")
        out.append("  }")
        return out

    def stage_out(dst, tile, lay, nb=64, nth=256):
        n4 = lay.QD // 4
        tot = nb * n4
        out = ["  { int cqo_ = cq; asm volatile(\"\" : \"+s\"(cqo_));"]
        for it in range(-(-tot // nth)):
            out.append(f"    {{ const int i_ = (int)threadIdx.x + {nth * it}, nl_ = i_ / {n4}, j_ = i_ - nl_ * {n4};")
            guard = f"i_ < {tot} && " if nth * (it + 1) > tot else ""
            out.append(f"      if ({guard}n0 + nl_ < n_nodes) {{ const float* t_ = {tile} + nl_ * {TP} + 4 * j_; "
                       f"*reinterpret_cast<float4*>({dst} + (size_t)(n0 + nl_) * {lay.row} + {_gofs(lay, 'j_')}) = "
                       "make_float4(t_[0], t_[1], t_[2], t_[3]); } }")
        out.append("  }")
        return out

    def cm_store(dst, tile, lay, nb, ind="  ", nth=256):
        """dst[(c * D + a) * n_nodes + n] = component a of channel c of node n, from a staged
        tile of nb nodes x the quad's 4 channels (coalesced nb-float runs per (c, a))"""
        dd = lay.D
        sh = nb.bit_length() - 1
        tot = Q * dd * nb

        def col():
            # LDS column of row r = cl * D + a: seg_start(a) + cl * d(a) + m(a), a select chain
            expr = None
            for (s0, s1, o, d) in lay.segs:
                a0 = s0 // 4                       # first component of this l-block
                v = f"{s0} + cl_ * {d} + (a_ - {a0})"
                expr = v if expr is None else f"(a_ >= {a0} ? {v} : {expr})"
            return expr
        # a rolled loop: its per-row address arithmetic stays inside (unrolled, the uniform row
        # values were hoisted to the kernel top and spilled SGPRs in grad-x).  Four consecutive
        # nodes per iteration leave as one float4 when the rows are 16-B aligned (n_nodes % 4 == 0,
        # the tile start is a multiple of 64): round 5, a quarter of the store instructions
        q4 = nb // 4
        sh4 = q4.bit_length() - 1
        out = ["{ int tid_ = threadIdx.x; asm volatile(\"\" : \"+v\"(tid_));",
               "  const bool v4_ = (n_nodes & 3) == 0;",
               "#pragma unroll 1",
               f"  for (int i_ = tid_; i_ < {tot // 4}; i_ += {nth}) {{",
               f"    const int row_ = i_ >> {sh4}, nl_ = (i_ & {q4 - 1}) * 4;",
               f"    const int cl_ = row_ / {dd}, a_ = row_ - cl_ * {dd};",
               f"    const int c_ = {col()};",
               f"    float* __restrict__ d_ = {dst} + (size_t)((cq * {Q} + cl_) * {dd} + a_) * n_nodes + n0 + nl_;",
               f"    const float t0_ = {tile}[nl_ * {TP} + c_], t1_ = {tile}[(nl_ + 1) * {TP} + c_],",
               f"                t2_ = {tile}[(nl_ + 2) * {TP} + c_], t3_ = {tile}[(nl_ + 3) * {TP} + c_];",
               "    if (v4_ && n0 + nl_ + 3 < n_nodes) {",
               "      *reinterpret_cast<float4*>(d_) = make_float4(t0_, t1_, t2_, t3_);",
               "    } else {",
               "      if (n0 + nl_ < n_nodes) d_[0] = t0_;",
               "      if (n0 + nl_ + 1 < n_nodes) d_[1] = t1_;",
               "      if (n0 + nl_ + 2 < n_nodes) d_[2] = t2_;",
               "      if (n0 + nl_ + 3 < n_nodes) d_[3] = t3_;",
               "    }",
               "  }", "}"]
        assert tot % 4 == 0 and nb % 4 == 0
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

    # block id -> (node tile, channel quad): the MUL / 4 quad workgroups of one node tile run on
    # one XCD (blockIdx % 8), so the lines of the tile's rows that several quads share (a quad
    # owns a 16*d-byte run of each 128*d-byte l-block) are fetched from HBM once, into that
    # XCD's L2, and its partial-line stores merge there
    NQ = MUL // Q
    def tile_map(nb):
        return ["  const int xcd = blockIdx.x & 7, rest_ = blockIdx.x >> 3;",
                f"  const int cq = rest_ % {NQ};",
                f"  const int n0 = ((rest_ / {NQ}) * 8 + xcd) * {nb};",
                "  if (n0 >= n_nodes) return;   // uniform per workgroup (tile count padded to 8)"]
    nrow = "lane" if SC_NT == 1 else "((wv >> 2) * 64 + lane)"   # this lane's node row in the tile
    head = tile_map(NB) + [
            "  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;",
            f"  const int c = __builtin_amdgcn_readfirstlane(cq * {Q} + (wv & {Q - 1}));",
            f"  const int cl = __builtin_amdgcn_readfirstlane(wv & {Q - 1});",
            f"  const float* __restrict__ cf = coef + (size_t)c * {cld};"]

    if SC_PK:
        emit_sc_packed(L, name, plan, lin, lout, D, Dout, TP, NB, NTH, head, stage_in, stage_out,
                       cm_store, lq)
    else:
        # ---------------- forward ----------------
        L.append(f"__global__ __launch_bounds__({NTH}) void sc_fwd_{name}(")
        L.append("    const float* __restrict__ x, const float* __restrict__ coef, int n_nodes,")
        L.append("    float* __restrict__ out) {")
        L.append(f"  __shared__ float tile[{NB} * {TP}];")
        L += head
        L += stage_in("x", "tile", lin, NB, NTH)
        L.append("  __syncthreads();")
        L.append(f"  float* __restrict__ tr = tile + {nrow} * {TP};")
        for a in range(D):
            L.append(f"  {VT} x{a} = {lds_get('tr', lq(lin, a, 'cl'))};")
        for q in range(Dout):
            L.append(f"  {VT} o{q} = {zero};")
        blocks = sc_blocks(plan, SC_BLOCK_FWD)
        fv = [f"x{a}" for a in range(D)] + [f"o{q}" for q in range(Dout)]
        pf = {}
        for j in range(min(SC_PFD_FWD, len(blocks))):
            lines, pf[j] = cload(blocks[j])
            L += lines
        for bi, blk in enumerate(blocks):
            # coefficients SC_PFD_FWD blocks ahead are in flight (scalar loads) while this block computes
            if bi + SC_PFD_FWD < len(blocks):
                lines, pf[bi + SC_PFD_FWD] = cload(blocks[bi + SC_PFD_FWD])
                L += lines
            nxt = [nm for j in range(bi + 1, bi + 1 + SC_PFD_FWD) for nm in pf.get(j, [])]
            carry = []
            if blk["kind"] == "deg1":
                for t, a, q in blk["deg1"]:
                    L.append(f"  o{q} = {cfma(t, f'x{a}', f'o{q}')};")
            for sg in blk.get("segs", []):
                a, b = sg["a"], sg["b"]
                pv = f"p{a}_{b}"
                if sg["first"]:
                    L.append(f"  {VT} {pv} = x{a} * x{b};")
                for t, q in sg["d2"]:
                    L.append(f"  o{q} = {cfma(t, pv, f'o{q}')};")
                for cc, lst in sg["d3"]:
                    L.append(f"  {{ const {VT} m = {pv} * x{cc};")
                    for t, q in lst:
                        L.append(f"    o{q} = {cfma(t, 'm', f'o{q}')};")
                    L.append("  }")
                if not sg["last"]:
                    carry = [pv]
            L.append("  " + pin(fv + carry, sgprs=nxt))
        L.append("  __syncthreads();")
        for q in range(Dout):
            L.append(f"  {lds_put('tr', lq(lout, q, 'cl'), f'o{q}')}")
        L.append("  __syncthreads();")
        L += stage_out("out", "tile", lout, NB, NTH)
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
        L.append(f"  float* __restrict__ xr = tx + {nrow} * {TP};")
        for a in range(D):
            L.append(f"  {VT} x{a} = {lds_get('xr', lq(lin, a, 'cl'))};")
            L.append(f"  {VT} d{a} = {zero};")
        L.append("  __syncthreads();")
        L += stage_in("gout", "tx", lout, NB, NTH)
        L.append("  __syncthreads();")
        L.append("  if (gt) {")
        L += cm_store("gt", "tx", lout, NB, "    ", NTH)
        L.append("  }")
        for q in range(Dout):
            L.append(f"  {VT} g{q} = {lds_get('xr', lq(lout, q, 'cl'))};")
        bv = [f"x{a}" for a in range(D)] + [f"g{q}" for q in range(Dout)] + [f"d{a}" for a in range(D)]
        blocks = sc_blocks(plan, SC_BLOCK_BWD)
        pf = {}
        for j in range(min(SC_PFD_BWD, len(blocks))):
            lines, pf[j] = cload(blocks[j])
            L += lines
        for bi, blk in enumerate(blocks):
            # coefficients SC_PFD_BWD blocks ahead are in flight (scalar loads) while this block computes
            if bi + SC_PFD_BWD < len(blocks):
                lines, pf[bi + SC_PFD_BWD] = cload(blocks[bi + SC_PFD_BWD])
                L += lines
            nxt = [nm for j in range(bi + 1, bi + 1 + SC_PFD_BWD) for nm in pf.get(j, [])]
            carry = []
            if blk["kind"] == "deg1":
                for t, a, q in blk["deg1"]:
                    L.append(f"  d{a} = {cfma(t, f'g{q}', f'd{a}')};")
            for sg in blk.get("segs", []):
                a, b = sg["a"], sg["b"]
                pv, sv = f"p{a}_{b}", f"s{a}_{b}"
                if sg["first"]:
                    L.append(f"  {VT} {pv} = x{a} * x{b}; {VT} {sv} = {zero};")
                for t, q in sg["d2"]:
                    L.append(f"  {sv} = {cfma(t, f'g{q}', sv)};")
                for cc, lst in sg["d3"]:
                    L.append(f"  {{ {VT} s = {zero};")
                    for t, q in lst:
                        L.append(f"    s = {cfma(t, f'g{q}', 's')};")
                    L.append(f"    d{cc} = {vfma('s', pv, f'd{cc}')}; {sv} = {vfma('s', f'x{cc}', sv)}; }}")
                if sg["last"]:
                    L.append(f"  d{a} = {vfma(sv, f'x{b}', f'd{a}')}; d{b} = {vfma(sv, f'x{a}', f'd{b}')};")
                else:
                    carry = [pv, sv]
            L.append("  " + pin(bv + carry, sgprs=nxt))
        L.append("  __syncthreads();")
        for a in range(D):
            L.append(f"  {lds_put('xr', lq(lin, a, 'cl'), f'd{a}')}")
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
        L.extend(tile_map(64))
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
    gpw = -(-nt // (WV * SC_COEF_MAXJG))      # term groups per wave
    JG = -(-nt // (WV * gpw))                 # terms per group (<= 64)
    assert JG <= 64 and NCB % 64 == 0
    if SC_COEF_CLUSTER:
        groups = coef_groups(plan, WV, JG, WV * gpw)
    else:
        groups = [list(range(s, min(s + JG, nt))) for s in range(0, nt, JG)]
    # lane j of group g ends with the sum of term perm[g * 64 + j] (-1: no term)
    perm = [(grp[j] if j < len(grp) else -1) for grp in groups for j in range(64)]
    nsub = NCB // 64
    NC4 = NCB // 4
    L.append(f"// coefficient gradient: {sum(1 for g in groups if g)} term groups of <= {JG} terms, {gpw} per wave;")
    L.append(f"// one workgroup = one channel x {NCB} LDS-resident nodes")
    L.append(f"__device__ const short sc_coef_perm_{name}[{len(perm)}] = {{")
    for k in range(0, len(perm), 32):
        L.append("  " + ", ".join(str(v) for v in perm[k: k + 32]) + ",")
    L.append("};")
    L.append(f"__global__ __launch_bounds__({64 * WV}) void sc_bwd_coef_{name}(")
    L.append("    const float* __restrict__ xt, const float* __restrict__ gt, int n_nodes, int chunk,")
    L.append("    float* __restrict__ part) {")
    SXS = NCB
    L.append(f"  __shared__ float sx[{D} * {NCB}];")
    L.append(f"  __shared__ float sg[{Dout} * {NCB}];")
    L.append("  const int ch = blockIdx.x, c = blockIdx.y;")
    L.append(f"  const int nb = ch * {NCB};")
    L.append(f"  const int cnt = min({NCB}, n_nodes - nb);")
    L.append("  const bool vec = (n_nodes & 3) == 0;")
    # whole aligned chunks (all but a ragged last one): every float4 load of a thread issued
    # before its first LDS store, one memory round trip; a clamped tail thread rewrites the
    # last float4 with the same value
    tot4 = (D + Dout) * NC4
    it_n = -(-tot4 // (64 * WV))

    def src_row(i):
        return (f"(a{i} < {D} ? xt + ((size_t)c * {D} + a{i}) * n_nodes : "
                f"gt + ((size_t)c * {Dout} + (a{i} - {D})) * n_nodes)")
    L.append(f"  if (vec && cnt == {NCB}) {{")
    for it in range(it_n):
        L.append(f"    const int i{it} = min((int)threadIdx.x + {64 * WV * it}, {tot4 - 1}), "
                 f"a{it} = i{it} / {NC4}, j{it} = 4 * (i{it} - a{it} * {NC4});")
        L.append(f"    const float4 v{it} = *reinterpret_cast<const float4*>({src_row(it)} + nb + j{it});")
    for it in range(it_n):
        L.append(f"    *reinterpret_cast<float4*>(a{it} < {D} ? sx + a{it} * {NCB} + j{it} : "
                 f"sg + (a{it} - {D}) * {NCB} + j{it}) = v{it};")
    L.append("  } else {")
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
    L.append("  }")
    L.append("  __syncthreads();")
    L.append("  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;")
    L.append(f"  float* __restrict__ dst = part + ((size_t)ch * {MUL} + c) * {cld};")
    L.append(f"  for (int k = 0; k < {gpw}; ++k) {{")
    L.append(f"    const int jg = __builtin_amdgcn_readfirstlane(k * {WV} + wv);")
    L.append("    float acc[64];")
    L.append("#pragma unroll")
    L.append("    for (int i = 0; i < 64; ++i) acc[i] = 0.0f;")
    L.append("    switch (jg) {")
    for gi, grp in enumerate(groups):
        if not grp:
            continue
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
        L.append("#pragma unroll 1")
        L.append(f"      for (int sb = 0; sb < {nsub}; ++sb) {{")
        L.append("        const int o = sb * 64 + lane;")
        for a in sorted(need_x):
            L.append(f"        const float x{a} = sx[{a * SXS} + o];")
        for q in sorted(need_g):
            L.append(f"        const float g{q} = sg[{q * SXS} + o];")
        # accumulator jj belongs to term grp[jj]; walk the terms by (a, b, c) so each pair
        # product and each triple product is formed once per group
        order = sorted(range(len(grp)), key=lambda jj: (plan.terms[grp[jj]][0] > 1,) + plan.terms[grp[jj]][1])
        cur, curc = None, None
        for jj in order:
            t = grp[jj]
            nu, (a, b, cc), q = plan.terms[t]
            if nu == 1:
                L.append(f"        acc[{jj}] = fmaf(x{a}, g{q}, acc[{jj}]);")
                continue
            if cur != (a, b):
                if cur is not None:
                    L.append("        }")
                    L.append("        " + cpin)
                L.append(f"        {{ const float p = x{a} * x{b};")
                cur, curc = (a, b), None
            if nu == 2:
                L.append(f"          acc[{jj}] = fmaf(p, g{q}, acc[{jj}]);")
            else:
                if curc != cc:
                    L.append(f"          const float m{cc} = p * x{cc};")
                    curc = cc
                L.append(f"          acc[{jj}] = fmaf(m{cc}, g{q}, acc[{jj}]);")
        if cur is not None:
            L.append("        }")
        L.append("        " + cpin)
        L.append("      }")
        L.append("      break; }")
    L.append("    default: break;")
    L.append("    }")
    L.append("    eelg_lane_reduce64(acc);")
    L.append(f"    const int t = jg < {len(groups)} ? sc_coef_perm_{name}[jg * 64 + lane] : -1;")
    L.append("    if (t >= 0) dst[t] = acc[0];")
    L.append("  }")
    L.append("}")
    WPB, NBC = WV, NCB
    cstream = 0
    csets = 0
    if SC_COEF_STREAM:
        code, csets = emit_sc_coef_stream(name, plan, D, Dout, cld)
        L += code
        cstream, NBC = 1, SC_COEF_SC
    info = dict(D=D, Dout=Dout, drow=drow, orow=orow, nterms=nt, cld=cld, njg=len(groups), wpb=WPB, nbc=NBC, nb=NB, nth=NTH,
                cmajor_out=cmajor_out, cstream=cstream, csets=csets,
                sig=fnv1a64(sc_signature(coupling, ls, corr)))
    return "\n".join(L), info


def emit_sc_coef_stream(name: str, plan, D: int, Dout: int, cld: int) -> Tuple[List[str], int]:
    """Streaming coefficient gradient ``sc_bwd_coefs_<name>`` (round 6).

    grad coef[c, t] = sum_n g_q(n) x_a(n) x_b(n) x_c(n) over the channel-major rows
    xt[(c D + a) N + n] / gt[(c Dout + q) N + n].  A workgroup of 16 waves owns one tile
    (channel c, node range r) and one of S term-group sets; wave w accumulates group s * 16 + w
    (<= 64 terms, one lane per node of a 64-node sub-tile) over every node of the range, so its
    accumulators are zeroed once and reduced across the 64 lanes once (eelg_lane_reduce64).

    The range streams through three LDS buffers of SC nodes filled by LDS-DMA two chunks ahead
    (no registers): each step opens with a counted ``vmcnt`` (this wave's DMA of the current
    chunk retired, the next chunk's still in flight) and a raw ``s_barrier`` (a
    ``__syncthreads()`` would drain every DMA); the buffer the step restages was last read before
    that barrier, its reads retired by their own ``lgkmcnt``.  Operand reads are inline asm (so
    hipcc does not drain the in-flight DMA before them), issued in the order the terms first use
    them, each waited for by a counted ``lgkmcnt`` just before its first use.
    SC_COEF_PAIRS (round 6): the image is [row pair][node][2] -- rows 2p and 2p + 1 of a node side
    by side -- so one ``ds_read_b64`` (2 LDS cycles) returns two operands, where the row image
    needed a ``ds_read2st64_b32`` (4 cycles); the pairs are filled by 4-byte LDS-DMA, 32 nodes x
    2 rows per wave-instruction (per-lane source offset fixed per workgroup).  An odd row count
    pads its last pair with a copy of its first row (never read).
    A chunk that passes the range's end, or rows that are not 16-B aligned (N % 4 != 0), are
    staged through registers with zero fill.  Blocks: the S set-blocks of a tile are consecutive
    on one XCD (their rows cross HBM once, then come from that XCD's L2).  part[r, c, t]: one
    deterministic partial per range."""
    WV, SC = 16, SC_COEF_SC
    PAIRS = SC_COEF_PAIRS
    PK = SC_COEF_PK and not PAIRS
    nt = len(plan.terms)
    S = -(-nt // (WV * (SC_COEF_PK_JG if PK else SC_COEF_MAXJG)))
    JG = -(-nt // (WV * S))
    assert JG <= (32 if PK else 64)
    groups = coef_sets(plan, S, WV, JG)
    ROWS = D + Dout
    NBUF = 3
    PX, PG = -(-D // 2), -(-Dout // 2)        # row pairs of x and of g (PAIRS)
    if PAIRS:
        NP = PX + PG
        BUFF = NP * SC * 2                     # floats per buffer
        NINS = NP * (SC // 32)                 # 4-byte DMA instructions per chunk (32 nodes x 2 rows)
        PB = SC * 8                            # bytes per pair block
        assert (NP - 1) * PB + (SC // 64 - 1) * 512 <= 65535
        NW = -(-NINS // WV)
    else:
        BUFF = ROWS * SC
        RB = SC * 4                            # bytes per LDS row (one wave-instruction)
        assert RB == 1024 and (ROWS - 1) * (RB // 256) + SC // 64 - 1 <= 255
        NW = -(-ROWS // WV)                    # most DMA rows a wave issues per chunk
    assert NBUF * BUFF * 4 <= 163840
    perm = [(grp[j] if j < len(grp) else -1) for grp in groups for j in range(64)]
    L: List[str] = []
    L.append(f"// streaming coefficient gradient: {S} sets x {WV} term groups of <= {JG} terms, "
             f"{SC}-node chunks, {'row-pair' if PAIRS else 'row'} image{', two nodes per lane' if PK else ''}")
    L.append(f"__device__ const short sc_coefs_perm_{name}[{len(perm)}] = {{")
    for k in range(0, len(perm), 32):
        L.append("  " + ", ".join(str(v) for v in perm[k: k + 32]) + ",")
    L.append("};")
    L.append(f"__global__ __launch_bounds__({64 * WV}) void sc_bwd_coefs_{name}(")
    L.append("    const float* __restrict__ xt, const float* __restrict__ gt, int n_nodes, int rn,")
    L.append("    float* __restrict__ part) {")
    L.append(f"  __shared__ __attribute__((aligned(16))) float sb_[{NBUF * BUFF}];")
    L.append("  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;")
    L.append("  const int nr = (n_nodes + rn - 1) / rn;             // node ranges (partial rows)")
    L.append(f"  const int q = blockIdx.x >> 3, st = q % {S};")
    L.append("  const int tile = (q / " + str(S) + ") * 8 + (blockIdx.x & 7);")
    L.append(f"  if (tile >= {MUL} * nr) return;                      // block-uniform")
    L.append("  const int c = tile / nr, r = tile - c * nr;")
    L.append("  const int nb0 = r * rn, nb1 = min(nb0 + rn, n_nodes);")
    L.append(f"  const int jg = st * {WV} + wv;")
    L.append("  const bool vec = (n_nodes & 3) == 0;")
    L.append(f"  const float* __restrict__ xr = xt + (size_t)c * {D} * n_nodes;")
    L.append(f"  const float* __restrict__ gr = gt + (size_t)c * {Dout} * n_nodes;")
    L.append("  const unsigned lds0 = (unsigned)(size_t)((__attribute__((address_space(3))) float*)sb_);")
    if PAIRS:
        # DMA instruction i = wv + 16 k of a chunk moves pair i / NB32, node block i % NB32; with
        # NB32 = 8 a wave keeps node block nb = wv & 7 and walks pairs h, h + 2, ... (h = wv >> 3).
        # Lane l: node 32 nb + l / 2 of row 2p + l % 2 (its element offset lo2, fixed per wave);
        # the pad row of an odd array repeats row 2p (lo1: in bounds, never read)
        assert SC // 32 == 8 and WV == 16
        L.append("  const int h = wv >> 3, nbk = wv & 7;")
        L.append("  const int lo2 = (lane & 1) * n_nodes + nbk * 32 + (lane >> 1), lo1 = nbk * 32 + (lane >> 1);")
    # stage(b, n0): chunk n0 into buffer b; returns the LDS-DMA instructions this wave issued
    L.append("  auto stage = [&](int b, int n0) -> int {")
    L.append("    if (n0 >= nb1) return 0;")
    L.append(f"    float* __restrict__ dst = sb_ + b * {BUFF};")
    L.append(f"    if (vec && n0 + {SC} <= nb1) {{")
    L.append("      int k = 0;")
    if PAIRS:
        # x pairs then g pairs, each a pointer stepping by 2 pairs (4 rows); pads only at the end
        for (arr, P0, P1, DD, off) in (("xr", 0, PX, D, 0), ("gr", PX, PX + PG, Dout, PX)):
            L.append(f"      {{ int pp = {P0} + ((h - {P0}) & 1);          // the first pair >= {P0} of this wave's parity")
            L.append(f"        const float* sp = {arr} + (size_t)(2 * (pp - {off})) * n_nodes + n0;")
            L.append(f"        for (; pp < {P1}; pp += 2, sp += (size_t)4 * n_nodes, ++k) {{")
            last_pad = DD % 2 == 1
            lo = f"(pp == {P1 - 1} ? lo1 : lo2)" if last_pad else "lo2"
            L.append(f"          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sp + {lo}),")
            L.append(f"              (__attribute__((address_space(3))) void*)(dst + pp * {SC * 2} + nbk * 64), 4, 0, 0);")
            L.append("        }")
            L.append("      }")
    else:
        L.append(f"      for (int row = wv; row < {ROWS}; row += {WV}, ++k) {{   // wave-uniform")
        L.append(f"        const float* src = (row < {D} ? xr + (size_t)row * n_nodes : gr + (size_t)(row - {D}) * n_nodes) + n0 + lane * 4;")
        L.append("        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,")
        L.append(f"            (__attribute__((address_space(3))) void*)(dst + row * {SC}), 16, 0, 0);")
    if not PAIRS:
        L.append("      }")
    L.append("      return k;")
    L.append("    } else {")
    L.append(f"      for (int i = threadIdx.x; i < {BUFF}; i += {64 * WV}) {{")
    if PAIRS:
        L.append(f"        const int pp = i / {2 * SC}, j = (i - pp * {2 * SC}) >> 1, n = n0 + j;")
        L.append(f"        const bool isx = pp < {PX};")
        L.append(f"        const int row = 2 * (isx ? pp : pp - {PX}) + (i & 1);")
        L.append(f"        const bool ok = n < nb1 && row < (isx ? {D} : {Dout});")
        L.append("        dst[i] = ok ? (isx ? xr : gr)[(size_t)row * n_nodes + n] : 0.0f;")
    else:
        L.append(f"        const int row = i / {SC}, j = i - row * {SC}, n = n0 + j;")
        L.append(f"        const float* src = row < {D} ? xr + (size_t)row * n_nodes : gr + (size_t)(row - {D}) * n_nodes;")
        L.append("        dst[i] = n < nb1 ? src[n] : 0.0f;")
    L.append("      }")
    L.append('      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // stores done before the barrier')
    L.append("      return 0;")
    L.append("    }")
    L.append("  };")
    # counted wait: everything but this wave's ``p`` newest LDS-DMA instructions has landed
    L.append("  auto retire = [&](int p) {")
    for k in range(NW, 0, -1):
        L.append(f'    {"if" if k == NW else "else if"} (p >= {k}) asm volatile("s_waitcnt vmcnt({k})" ::: "memory");')
    L.append('    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
    L.append("  };")
    if PK:
        L.append(f"  eelg_f2r acc[{JG}];")
        L.append("#pragma unroll")
        L.append(f"  for (int i = 0; i < {JG}; ++i) acc[i] = (eelg_f2r){{0.0f, 0.0f}};")
    else:
        L.append("  float acc[64];")
        L.append("#pragma unroll")
        L.append("  for (int i = 0; i < 64; ++i) acc[i] = 0.0f;")
    L.append("  stage(0, nb0);")
    L.append(f"  int pend = stage(1, nb0 + {SC});           // this wave's DMAs of the chunk after the current")
    # the chunk loop sits inside each case: the accumulators never meet at a merge point inside
    # the loop (a switch inside the loop made the compiler move all 64 of them at every case exit
    # and spill); every wave, a group-less one too, runs the same stages and barriers
    lane_b = 8 if (PAIRS or PK) else 4       # bytes per lane of a sub-tile row read
    NST = 128 if PK else 64                  # nodes per sub-tile
    head = ["      int b = 0;",
            f"      for (int n0 = nb0; n0 < nb1; n0 += {SC}, b = b == {NBUF - 1} ? 0 : b + 1) {{",
            "        retire(pend);                         // chunk n0 landed (this wave's part)",
            '        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");',
            "        __builtin_amdgcn_s_barrier();        // every wave's part; the buffer restaged next is free",
            f"        pend = stage(b == 0 ? 2 : b - 1, n0 + {2 * SC});",
            f"        const unsigned ab = lds0 + b * {BUFF * 4} + lane * {lane_b};"]
    tail = ["      }",
            '      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");']
    L.append("  switch (jg) {")
    for gi, grp in enumerate(groups):
        if not grp:
            continue
        L.append(f"    case {gi}: {{")
        L += head
        cpin = pin([f"acc[{jj}]" for jj in range(len(grp))])
        L.append("#pragma unroll 1")
        L.append(f"      for (int sb = 0; sb < {SC // NST}; ++sb) {{")
        L.append(f"        const unsigned a_ = ab + sb * {64 * lane_b};")
        order = sorted(range(len(grp)), key=lambda jj: (plan.terms[grp[jj]][0] > 1,) + plan.terms[grp[jj]][1])
        seq = []
        for jj in order:
            nu, (a, b_, cc), qq = plan.terms[grp[jj]]
            for o in ([("x", a), ("g", qq)] if nu == 1 else
                      [("x", a), ("x", b_)] + ([("x", cc)] if nu == 3 else []) + [("g", qq)]):
                if o not in seq:
                    seq.append(o)
        if PAIRS:
            # a read = one row pair: (kind, pair) in first-use order; it yields both rows
            def pair_of(o):
                return (o[0], o[1] // 2)
            reads = []
            for o in seq:
                if pair_of(o) not in reads:
                    reads.append(pair_of(o))
            ridx = {o: reads.index(pair_of(o)) for o in seq}
            used = set(seq)
        elif PK:
            reads = [(o,) for o in seq]           # one row per read, two nodes
            ridx = {o: k for k, rd in enumerate(reads) for o in rd}
        else:
            reads = [tuple(seq[k: k + 2]) for k in range(0, len(seq), 2)]
            ridx = {o: k for k, rd in enumerate(reads) for o in rd}
        row = {o: (o[1] if o[0] == "x" else D + o[1]) for o in seq}
        VT = "eelg_f2r" if PK else "float"
        L.append(f"        {VT} " + ", ".join(f"{o[0]}{o[1]}" for o in seq) + ";")
        for k, rd in enumerate(reads):
            if PAIRS:
                kind, pp = rd
                blk = pp if kind == "x" else PX + pp
                L.append(f"        eelg_f2r p{k};")
                L.append(f'        asm volatile("ds_read_b64 %0, %1 offset:{blk * PB}" : "=v"(p{k}) : "v"(a_));')
            elif PK:
                L.append(f"        eelg_f2r p{k};")
                L.append(f'        asm volatile("ds_read_b64 %0, %1 offset:{row[rd[0]] * RB}" : "=v"(p{k}) : "v"(a_));')
            elif len(rd) == 2:
                L.append(f"        eelg_f2r p{k};")
                L.append(f'        asm volatile("ds_read2st64_b32 %0, %1 offset0:{row[rd[0]] * (RB // 256)} '
                         f'offset1:{row[rd[1]] * (RB // 256)}" : "=v"(p{k}) : "v"(a_));')
            else:
                L.append(f"        float p{k};")
                L.append(f'        asm volatile("ds_read_b32 %0, %1 offset:{row[rd[0]] * RB}" : "=v"(p{k}) : "v"(a_));')
        state = {"w": -1}

        def need(*opsn):
            k = max(ridx[o] for o in opsn)
            if k <= state["w"]:
                return
            regs = [f"p{j}" for j in range(state["w"] + 1, k + 1)]
            # (the counter field holds 0..15: a larger count waits for more than this read)
            L.append(f'        asm volatile("s_waitcnt lgkmcnt({min(15, len(reads) - 1 - k)})" : ' +
                     ", ".join(f'"+v"({v})' for v in regs) + ' : : "memory");')
            for j in range(state["w"] + 1, k + 1):
                rd = reads[j]
                if PAIRS:
                    kind, pp = rd
                    parts = [f"{kind}{2 * pp + h} = p{j}[{h}];" for h in (0, 1) if (kind, 2 * pp + h) in used]
                    L.append("        " + " ".join(parts))
                elif PK:
                    L.append(f"        {rd[0][0]}{rd[0][1]} = p{j};")
                elif len(rd) == 2:
                    L.append(f"        {rd[0][0]}{rd[0][1]} = p{j}[0]; {rd[1][0]}{rd[1][1]} = p{j}[1];")
                else:
                    L.append(f"        {rd[0][0]}{rd[0][1]} = p{j};")
            state["w"] = k
        cur, curc = None, None
        for jj in order:
            t = grp[jj]
            nu, (a, b_, cc), qq = plan.terms[t]
            FMA = (lambda u, v, w: f"__builtin_elementwise_fma({u}, {v}, {w})") if PK else \
                (lambda u, v, w: f"fmaf({u}, {v}, {w})")
            if nu == 1:
                need(("x", a), ("g", qq))
                L.append(f"        acc[{jj}] = {FMA(f'x{a}', f'g{qq}', f'acc[{jj}]')};")
                continue
            if cur != (a, b_):
                if cur is not None:
                    L.append("        }")
                    L.append("        " + cpin)
                need(("x", a), ("x", b_))
                L.append(f"        {{ const {VT} pp = x{a} * x{b_};")
                cur, curc = (a, b_), None
            if nu == 2:
                need(("g", qq))
                L.append(f"          acc[{jj}] = {FMA('pp', f'g{qq}', f'acc[{jj}]')};")
            else:
                if curc != cc:
                    need(("x", cc))
                    L.append(f"          const {VT} m{cc} = pp * x{cc};")
                    curc = cc
                need(("g", qq))
                L.append(f"          acc[{jj}] = {FMA(f'm{cc}', f'g{qq}', f'acc[{jj}]')};")
        if cur is not None:
            L.append("        }")
        L.append("        " + cpin)
        L.append("      }")
        L += tail
        L.append("      break; }")
    L.append("    default: {")
    L += [ln for ln in head if "const unsigned ab" not in ln] + tail
    L.append("      break; }")
    L.append("  }")
    if PK:
        # the two nodes of each lane first, then the 64 lanes
        L.append("  float red[64];")
        L.append("#pragma unroll")
        L.append(f"  for (int i = 0; i < 64; ++i) red[i] = i < {JG} ? acc[i < {JG} ? i : 0][0] + acc[i < {JG} ? i : 0][1] : 0.0f;")
        L.append("  eelg_lane_reduce64(red);")
        L.append(f"  const int t = sc_coefs_perm_{name}[jg * 64 + lane];")
        L.append(f"  if (t >= 0) part[((size_t)r * {MUL} + c) * {cld} + t] = red[0];")
    else:
        L.append("  eelg_lane_reduce64(acc);")
        L.append(f"  const int t = sc_coefs_perm_{name}[jg * 64 + lane];")
        L.append(f"  if (t >= 0) part[((size_t)r * {MUL} + c) * {cld} + t] = acc[0];")
    L.append("}")
    return L, S


# ---------------------------------------------------------------------------
def main(outdir: str) -> None:
    os.makedirs(outdir, exist_ok=True)
    global _PKV
    _PKV = "volatile" if SC_PK_SCHED else ""
    parts = ["// GENERATED by csrc/gen_kernels.py -- do not edit", "#include <hip/hip_runtime.h>",
             "#include <stdint.h>", '#include "../eelg_internal.h"', "",
             "// dword-aligned vector types: per-lane runs of d floats start at 4-byte boundaries",
             "typedef float eelg_f4u __attribute__((ext_vector_type(4), aligned(4)));",
             "typedef float eelg_f3u __attribute__((ext_vector_type(3), aligned(4)));",
             "typedef float eelg_f2u __attribute__((ext_vector_type(2), aligned(4)));",
             "typedef float eelg_f4a __attribute__((ext_vector_type(4)));",
             "typedef float eelg_f4r __attribute__((ext_vector_type(4)));",
             "// SGPR coefficient vectors of the contraction (dword-aligned scalar loads)",
             "typedef float eelg_c2 __attribute__((ext_vector_type(2), aligned(4)));",
             "typedef float eelg_c4 __attribute__((ext_vector_type(4), aligned(4)));",
             "typedef float eelg_c8 __attribute__((ext_vector_type(8), aligned(4)));",
             "typedef float eelg_c16 __attribute__((ext_vector_type(16), aligned(4)));",
             "typedef float eelg_f2r __attribute__((ext_vector_type(2)));",
             "// packed contraction: acc (two nodes) += / = coefficient x b, the coefficient broadcast from",
             "// the low / high half of an aligned SGPR pair by op_sel / op_sel_hi",
             f'#define EELG_PKF_LO(acc, cp, b) asm {_PKV}("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "s"(cp), "v"(b))',
             f'#define EELG_PKF_HI(acc, cp, b) asm {_PKV}("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(cp), "v"(b))',
             # the first term of a sum: an FMA onto the inline constant 0, not a v_pk_mul with op_sel
             # (a VOP3P multiply with a broadcast operand costs its reader an s_nop)
             f'#define EELG_PKM_LO(acc, cp, b) asm {_PKV}("v_pk_fma_f32 %0, %1, %2, 0 op_sel_hi:[0,1,1]" : "=v"(acc) : "s"(cp), "v"(b))',
             f'#define EELG_PKM_HI(acc, cp, b) asm {_PKV}("v_pk_fma_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "=v"(acc) : "s"(cp), "v"(b))',
             ('#define EELG_PKMV(d, a, b) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))'
              if SC_PK_SCHED else '#define EELG_PKMV(d, a, b) ((d) = (a) * (b))'),
             ('#define EELG_PKFV(d, a, b) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b))'
              if SC_PK_SCHED else '#define EELG_PKFV(d, a, b) ((d) = __builtin_elementwise_fma((a), (b), (d)))'),
             "template <typename V> __device__ __forceinline__ eelg_f2r eelg_splat(V v, int i) {",
             "  return (eelg_f2r){v[i], v[i]};",
             "}",
             "template <typename V> __device__ __forceinline__ eelg_f2r eelg_pair(V v, int j) {",
             "  return (eelg_f2r){v[2 * j], v[2 * j + 1]};",
             "}", ""]
    header = parts
    global MUL
    for mul in kernel_sets.MULS:
        MUL = mul
        sfx = "" if mul == 32 else f"_m{mul}"
        parts = list(header)
        if mul == 32:
            for lmax in kernel_sets.LMAX:
                parts.append(emit_sh(lmax))
        # the row a tp_fwd stream reads for an edge past its range (also when the batch has no
        # edges and the edge tensors are empty): as long as the longest x / SH / weight row
        pad = max(max(node.dim, (sh.dim + 3) // 4 * 4, sum(p.mul for p in cg.tp_paths(node, sh, target)))
                  for node, sh, target in tp_configs().values())
        parts.append(f"static __device__ __attribute__((aligned(16))) float eelg_tp_pad[{(pad + 3) // 4 * 4}];\n")
        tp_table, sc_table = [], []
        # bf16 storage of the edge tensors (BASELINE config 5) is generated for mul = 32 only
        bf = mul == 32
        for name, (node, sh, target) in tp_configs().items():
            code, info = emit_tp(name + sfx, node, sh, target)
            parts.append(code)
            info["ngroups_bf"] = 0
            if bf:
                code_bf, info_bf = emit_tp(name + sfx, node, sh, target, "bf16")
                parts.append(code_bf)
                info["ngroups_bf"] = info_bf["ngroups"]
            tp_table.append((name + sfx, info))
        for name, (coupling, ls, corr) in sc_configs().items():
            code, info = emit_sc(name + sfx, coupling, ls, corr)
            parts.append(code)
            sc_table.append((name + sfx, info))
        # launch tables
        parts.append("\n// ===== config tables =====")
        parts.append(f"static const eelg_tp_cfg kTpConfigs[] = {{")
        for name, i in tp_table:
            lmax = int(name.split("_l")[1].split("_")[0])
            bfk = (f"tp_fwd_{name}_bw, tp_bwd_{name}_bw, tp_bws_{name}, tp_bws_{name}_bw" if bf
                   else f"nullptr, nullptr, tp_bws_{name}, nullptr")
            bwk = (f"tp_bwf_{name}, " + (f"tp_bwf_{name}_bw" if bf else "nullptr")) if i["bwf"] else "nullptr, nullptr"
            bws_ = f"bwf_slots_{name}, bwf_alpha_{name}" if i["bwf"] else "nullptr, nullptr"
            parts.append(f'  {{"{name}", {i["din"]}, {i["dmid"]}, {i["wn"]}, {i["nsh"]}, {i["ngroups"]}, '
                         f'{i["npaths"]}, {lmax}, {i["nbgroups"]}, {i["nph"]}, {i["beph"]}, {i["fwpb"]}, 0x{i["sig"]:016x}ULL, tp_fwd_{name}, tp_bwd_{name}, '
                         f'{bfk}, {i["ngroups_bf"]}, {i["bxcd"]}, {bwk}, {i["bwf_r"]}, {i["tdim"]}, {bws_}}},')
        parts.append("};")
        parts.append("static const eelg_sc_cfg kScConfigs[] = {")
        for name, i in sc_table:
            parts.append(f'  {{"{name}", {i["D"]}, {i["Dout"]}, {i["drow"]}, {i["orow"]}, {i["nterms"]}, {i["njg"]}, {i["wpb"]}, '
                         f'0x{i["sig"]:016x}ULL, sc_fwd_{name}, sc_bwd_x_{name}, sc_bwd_coef_{name}, sc_cmajor_{name}, '
                         f'{i["cmajor_out"]}, {i["nbc"]}, {i["nb"]}, {i["nth"]}, {i["cld"]}, '
                         f'{"sc_bwd_coefs_" + name if i["cstream"] else "nullptr"}, {i["csets"]}}},')
        parts.append("};")
        parts.append(f"const eelg_tp_cfg* eelg_tp_table_m{mul}(int* n) {{ *n = (int)(sizeof(kTpConfigs)/sizeof(kTpConfigs[0])); return kTpConfigs; }}")
        parts.append(f"const eelg_sc_cfg* eelg_sc_table_m{mul}(int* n) {{ *n = (int)(sizeof(kScConfigs)/sizeof(kScConfigs[0])); return kScConfigs; }}")
        src = "\n".join(parts) + "\n"
        path = os.path.join(outdir, f"eelg_gen{sfx}.hip")
        old = open(path).read() if os.path.exists(path) else None
        if old != src:
            with open(path, "w") as f:
                f.write(src)
        print(f"wrote {path}: {len(src.splitlines())} lines")
    MUL = kernel_sets.MUL


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "generated"))
