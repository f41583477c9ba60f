#!/usr/bin/env python3
"""Per-kernel micro-benchmark at the bench shapes (32 graphs x 1024 nodes / 4096 edges).

Times every hot-path op in isolation with HIP events (median of reps) and prints
algorithmic bytes / FLOPs and the implied rates.  Usage: python tools/kbench.py [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd"))

import torch  # noqa: E402

from gnn import ops  # noqa: E402
from gnn.data import collate  # noqa: E402
from gnn.synthetic import SyntheticLattices  # noqa: E402
from gnn.o3 import Linear  # noqa: E402
from gnn.mace import SymmetricContraction  # noqa: E402
from gnn.blocks import TensorProductInteractionBlock  # noqa: E402
from gnn.irreps import Irreps  # noqa: E402


ONLY = None


def _morton(d):
    """the same lattice with its nodes renumbered along a Morton (Z-order) curve"""
    import copy
    pos = d.positions
    lo, hi = pos.min(0).values, pos.max(0).values
    q = ((pos - lo) / (hi - lo).clamp_min(1e-12) * 1023).long().clamp(0, 1023)
    key = torch.zeros(pos.shape[0], dtype=torch.long)
    for bit in range(10):
        for ax in range(3):
            key |= ((q[:, ax] >> bit) & 1) << (3 * bit + ax)
    perm = torch.argsort(key)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    e = copy.copy(d)
    e.positions = pos[perm]
    e.node_attrs = d.node_attrs[perm]
    e.edge_index = inv[d.edge_index]
    return e


def timeit(fn, reps):
    if reps == 0:
        return float("nan")
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--graphs", type=int, default=32)
    ap.add_argument("--only", default="", help="regex: time only matching ops")
    ap.add_argument("--morton", action="store_true", help="renumber each graph's nodes in Morton order")
    args = ap.parse_args()
    dev = "cuda"
    ds = SyntheticLattices(args.graphs, 1024, 4096, 1234)
    graphs = [ds[g] for g in range(args.graphs)]
    if args.morton:
        graphs = [_morton(g) for g in graphs]
    b = collate(graphs).to(dev)
    n = b.node_attrs.shape[0]
    csr = ops.EdgeCSR.build(b.edge_index, n)
    e = csr.num_edges
    hid = "32x0e+32x1o+32x2e+32x3o+32x4e"
    sh_ir = Irreps.spherical_harmonics(4)
    res = {}

    import re as _re

    def want(name):
        return not args.only or _re.search(args.only, name)

    def timeit_if(name, fn, reps):
        return timeit(fn, reps) if want(name) else float("nan")

    def rec(name, ms, bytes_=None, flops=None):
        if not want(name):
            return
        r = {"ms": round(ms, 4)}
        if bytes_:
            r["GB/s"] = round(bytes_ / ms / 1e6, 1)
        if flops:
            r["TFLOP/s"] = round(flops / ms / 1e9, 2)
        res[name] = r
        print(f"{name:32s} {ms:8.4f} ms " + " ".join(f"{k}={v}" for k, v in r.items() if k != "ms"),
              flush=True)

    sh, feats = ops.edge_embed(b.positions, csr, b.shifts[csr.perm], b.edge_attr[csr.perm].reshape(-1),
                               4, 6, 0.6, 0.05)
    rec("edge_embed", timeit_if("edge_embed", lambda: ops.edge_embed(b.positions, csr, b.shifts[csr.perm],
                                                     b.edge_attr[csr.perm].reshape(-1), 4, 6, 0.6, 0.05),
                             args.reps))
    blk = TensorProductInteractionBlock(hid, sh_ir, "12x0e", hid, 4.0).to(dev)
    idx, info = blk._config()
    x = torch.randn(n, 800, device=dev)
    w = torch.randn(e, info["wn"], device=dev)
    agg = ops.tp_interaction(x, sh, w, csr, idx, info, 0.25)
    tp_bytes = 4 * (n * 800 + e * 25 + e * info["wn"] + e + n + 1 + n * info["dmid"])
    tp_flops = 2 * 32 * 1302 * e
    rec("tp_fwd (B)", timeit_if("tp_fwd (B)", lambda: ops.tp_interaction(x, sh, w, csr, idx, info, 0.25), args.reps),
        tp_bytes, tp_flops)
    g = torch.randn_like(agg)
    gw = torch.empty_like(w)
    gxe = torch.empty(e, 800, device=dev)
    lib = ops._lib.load()

    def tpb():
        ops._lib.check(lib.eelg_tp_bwd(idx, ops._lib.ptr(x), ops._lib.ptr(sh), ops._lib.ptr(w),
                                       ops._lib.ptr(csr.sender), ops._lib.ptr(csr.receiver), e,
                                       ops._lib.ptr(g), 0.25, ops._lib.ptr(gw), ops._lib.ptr(gxe),
                                       ops._lib.stream(x)), "tp_bwd")
    bwd_bytes = 4 * (n * 800 + e * 25 + 2 * e * info["wn"] + 2 * e + e * 800 + n * info["dmid"])
    rec("tp_bwd (B)", timeit_if("tp_bwd (B)", tpb, args.reps), bwd_bytes, 2 * tp_flops)
    # fused output-linear grad-x + TP backward (replaces lin 7360->800 bwd_x + tp_bwd)
    gyl = torch.randn(n, 800, device=dev)
    lw = blk.linear.weight.detach().contiguous()

    def tpbf():
        ops._lib.check(lib.eelg_tp_bwd_fused(idx, ops._lib.ptr(x), ops._lib.ptr(sh), ops._lib.ptr(w),
                                             ops._lib.ptr(csr.sender), ops._lib.ptr(csr.receiver),
                                             ops._lib.ptr(csr.rowptr), n,
                                             ops._lib.ptr(gyl), ops._lib.ptr(lw), 0.25, ops._lib.ptr(gw),
                                             ops._lib.ptr(gxe), ops._lib.stream(x)), "tp_bwf")
    bwf_bytes = 4 * (n * 800 + e * 25 + 2 * e * info["wn"] + 2 * e + e * 800 + n * 800 + n + 1)
    rec("tp_bwf (B, fused linear)", timeit_if("tp_bwf (B, fused linear)", tpbf, args.reps), bwf_bytes,
        2 * tp_flops + 2 * n * 7360 * 32)
    rec("segment_sum gxe->gx (800)", timeit_if("segment_sum gxe->gx (800)", lambda: ops.segment_sum_csr(gxe, csr.srowptr, n, idx=csr.sperm), args.reps),
        4 * (e * 800 + n * 800 + 2 * e))
    m7360 = torch.randn(e, 7360, device=dev)
    rec("segment_sum unfused (7360)", timeit_if("segment_sum unfused (7360)", lambda: ops.segment_sum_csr(m7360, csr.rowptr, n), args.reps),
        4 * (e * 7360 + n * 7360 + e))
    del m7360
    sc = SymmetricContraction(hid, hid, 3).to(dev)
    sidx, sinfo = sc._config()
    coef = sc.coefficients().detach()
    xs = torch.randn(n, 800, device=dev)
    nt = sinfo["nterms"]
    rec("sc_fwd", timeit_if("sc_fwd", lambda: ops.symmetric_contraction(xs, coef, sidx, sinfo, 32), args.reps),
        4 * 2 * n * 800, 2 * n * 32 * (nt + 3250))
    gs = torch.randn(n, 800, device=dev)
    gx = torch.empty_like(xs)

    def scbx():
        ops._lib.check(lib.eelg_sc_bwd_x(sidx, ops._lib.ptr(xs), ops._lib.ptr(coef), ops._lib.ptr(gs), n,
                                         32, ops._lib.ptr(gx), ops._lib.stream(x)), "bx")
    rec("sc_bwd_x", timeit_if("sc_bwd_x", scbx, args.reps), 4 * 3 * n * 800, 2 * n * 32 * (nt + 2 * 3250))
    xt = torch.empty(800, n, device=dev)
    gt = torch.empty(800, n, device=dev)

    def cm():
        ops._lib.check(lib.eelg_sc_cmajor(sidx, 0, ops._lib.ptr(xs), n, 32, ops._lib.ptr(xt),
                                          ops._lib.stream(x)), "cm")
    rec("sc_cmajor", timeit_if("sc_cmajor", cm, args.reps), 4 * 2 * n * 800)
    cm()
    ops._lib.check(lib.eelg_sc_cmajor(sidx, 1, ops._lib.ptr(gs), n, 32, ops._lib.ptr(gt), ops._lib.stream(x)), "cm")
    chunk = sinfo["coef_chunk"]                                     # as gnn/ops.py
    nch = int(lib.eelg_sc_bwd_coef_parts(sidx, n, 32))
    part = torch.empty(nch, 32, sinfo["coef_ld"], device=dev)

    def scbc():
        ops._lib.check(lib.eelg_sc_bwd_coef(sidx, ops._lib.ptr(xt), ops._lib.ptr(gt), n, 32, chunk,
                                            ops._lib.ptr(part), ops._lib.stream(x)), "bc")
    rec("sc_bwd_coef", timeit_if("sc_bwd_coef", scbc, args.reps), None, 2 * n * 32 * (nt + 3250))
    for name, ii, oo in [("lin 800->400 (readout, 16 ch)", hid, "16x0e+16x1o+16x2e+16x3o+16x4e"),
                         ("lin 800->800", hid, hid),
                         ("lin 7360->800", "160x0e+256x1o+320x2e+320x3o+288x4e", hid)]:
        lin = Linear(ii, oo).to(dev)
        xi = torch.randn(n, lin.irreps_in.dim, device=dev)
        gy = torch.randn(n, lin.irreps_out.dim, device=dev)
        byt = 4 * n * (lin.irreps_in.dim + lin.irreps_out.dim)
        fl = 2 * n * sum(lin.irreps_in[i].mul * lin.irreps_out[o].mul * lin.irreps_in[i].ir.dim
                         for i, o in lin.instructions)
        rec(f"{name} fwd", timeit_if(f"{name} fwd", lambda: lin._fwd(xi, lin.weight, None), args.reps), byt, fl)
        rec(f"{name} bwd_x", timeit_if(f"{name} bwd_x", lambda: lin._bwd_x(gy, lin.weight), args.reps), byt, fl)
        rec(f"{name} bwd_w", timeit_if(f"{name} bwd_w", lambda: lin._bwd_w(xi, gy), args.reps), byt, fl)
        if hasattr(lin, "_pk_cache"):
            def pack():
                lin._pk_cache.clear()
                lin._packed("fwd", lin.weight.detach())
            rec(f"{name} weight pack", timeit_if(f"{name} weight pack", pack, args.reps), None, None)
    mlp = blk.conv_tp_weights
    ef = torch.randn(e, 12, device=dev, requires_grad=True)
    efn = ef.detach()
    rad_fl = 2 * e * (12 * 64 + 64 * 64 + 64 * info["wn"])
    rec("radial fwd (HIP)", timeit_if("radial fwd (HIP)", lambda: ops.radial_mlp(efn, mlp), args.reps),
        None, rad_fl)

    def radfb():
        out = ops.radial_mlp(efn, mlp)
        out.backward(torch.ones_like(out))
    rec("radial fwd+bwd (HIP)", timeit_if("radial fwd+bwd (HIP)", radfb, args.reps), None, 3 * rad_fl)
    rec("radial MLP fwd (torch)", timeit_if("radial MLP fwd (torch)", lambda: mlp(ef), args.reps), None,
        2 * e * (12 * 64 + 64 * 64 + 64 * info["wn"]))

    def mlpfb():
        out = mlp(ef)
        out.backward(torch.ones_like(out))
    rec("radial MLP fwd+bwd (nn.Sequential)", timeit_if("radial MLP fwd+bwd (torch)", mlpfb, args.reps), None,
        3 * 2 * e * (12 * 64 + 64 * 64 + 64 * info["wn"]))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
