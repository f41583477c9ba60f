#!/usr/bin/env python3
"""Targeted check: single-slot multi-chunk irreps linear; which rows / which partial sums."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402


def main():
    from gnn.o3 import Linear
    for irin, irout, n in [("64x0e", "32x0e", 256), ("160x0e", "32x0e", 256), ("96x1o", "32x1o", 128)]:
        torch.manual_seed(0)
        m = Linear(irin, irout).cuda()
        x = torch.randn(n, m.irreps_in.dim, device="cuda")
        with torch.no_grad():
            y = m(x).double().cpu()
        K = m.irreps_in[0].mul
        d = m.irreps_in[0].ir.dim
        W = m.weight.detach().double().cpu().view(K, -1) / K ** 0.5
        xv = x.double().cpu().view(n, K, d)
        ref = torch.einsum("nkm,kj->njm", xv, W).reshape(n, -1)
        err = (y - ref).abs()
        bad_nodes = torch.nonzero(err.max(1).values > 1e-4).flatten().tolist()
        print(f"{irin}->{irout} n={n}: max err {err.max():.3e}; bad nodes {len(bad_nodes)}: {bad_nodes[:20]}")
        # per MFMA row within a 32-row tile
        rows = err.view(n, 32, d).permute(0, 2, 1).reshape(n * d, 32).max(1).values
        badr = torch.nonzero(rows > 1e-4).flatten()
        print("   bad rows mod 32:", sorted(set((badr % 32).tolist())))
        print("   bad rows mod 128 count:", len(set((badr % 128).tolist())))
        # is y equal to the partial sum missing some chunks?
        for c in range(1, (K + 31) // 32):
            part = torch.einsum("nkm,kj->njm", xv[:, : 32 * c], W[: 32 * c]).reshape(n, -1)
            e2 = (y - part).abs().view(n * d, 32)
            print(f"   rows equal to sum over first {c} chunk(s): {(e2.max(1).values < 1e-4).sum().item()} / {n * d}")


if __name__ == "__main__":
    main()
