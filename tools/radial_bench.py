"""Times the fused radial MLP (eelg_radial_fwd / eelg_radial_bwd) against the same MLP as
library GEMMs (torch addmm / hipBLASLt) at the bench shape: E = 131072 edges (32 graphs x
4096), 12 -> 64 -> 64 -> 1344.  HIP-event medians over --reps runs."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd"))
from gnn import ops  # noqa: E402


def timeit(fn, reps):
    ts = []
    for _ in range(reps + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edges", type=int, default=131072)
    ap.add_argument("--width", type=int, default=1344)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    e, w = a.edges, a.width
    torch.manual_seed(0)
    seq = torch.nn.Sequential(torch.nn.Linear(12, 64), torch.nn.SiLU(), torch.nn.Linear(64, 64),
                              torch.nn.SiLU(), torch.nn.Linear(64, w, bias=False)).cuda()
    feats = torch.rand(e, 12, device="cuda")
    g = torch.randn(e, w, device="cuda")
    flops = 2 * e * (12 * 64 + 64 * 64 + 64 * w)
    out_bytes = 4 * e * w

    def fused_fwd():
        return ops.radial_mlp(feats, seq)

    y = fused_fwd()
    t_f = timeit(fused_fwd, a.reps)

    def fused_bwd():
        seq.zero_grad(set_to_none=True)
        y.backward(g, retain_graph=True)
    t_b = timeit(fused_bwd, a.reps)

    def lib_fwd():
        return seq(feats)
    yl = lib_fwd()
    t_lf = timeit(lib_fwd, a.reps)

    def lib_bwd():
        seq.zero_grad(set_to_none=True)
        yl.backward(g, retain_graph=True)
    t_lb = timeit(lib_bwd, a.reps)
    print(f"radial MLP E={e} W={w}: fwd {flops / 1e9:.2f} GFLOP, writes {out_bytes / 1e6:.0f} MB")
    print(f"  fused fwd  {t_f:.3f} ms  ({flops / t_f / 1e9:.1f} TFLOP/s, {out_bytes / t_f / 1e6:.0f} GB/s)")
    print(f"  fused bwd  {t_b:.3f} ms  ({2 * flops / t_b / 1e9:.1f} TFLOP/s, reads grad_w twice)")
    print(f"  torch fwd  {t_lf:.3f} ms")
    print(f"  torch bwd  {t_lb:.3f} ms")


if __name__ == "__main__":
    main()
