#!/usr/bin/env python3
"""Per-piece check of the irreps linear kernels (fwd, grad-x, grad-W) against fp64 torch,
over the model's shapes and odd ones.  Prints one line per case; exits 1 on any failure."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd")]

import torch  # noqa: E402

CASES = [
    ("1x0e", "32x0e", False, 200),
    ("32x0e", "32x0e", False, 200),
    ("32x0e+32x1o+32x2e+32x3o+32x4e", "32x0e+32x1o+32x2e+32x3o+32x4e", False, 200),
    ("32x0e+32x1o+32x2e+32x3o+32x4e", "32x0e+32x1o+32x2e+32x3o+32x4e", False, 1000),
    ("160x0e+256x1o+320x2e+320x3o+288x4e", "32x0e+32x1o+32x2e+32x3o+32x4e", True, 200),
    ("160x0e+256x1o+320x2e+320x3o+288x4e", "32x0e+32x1o+32x2e+32x3o+32x4e", True, 333),
    ("32x0e+32x1o+32x2e+32x3o+32x4e", "160x0e+32x1o+32x2e+32x3o+32x4e", False, 257),
    ("32x0e+32x1o+32x2e+32x3o+32x4e", "16x0e+16x1o+16x2e+16x3o+16x4e", False, 200),
    ("16x0e+16x1o+16x2e+16x3o+16x4e", "2x0e+2x2e+1x4e", True, 5),
    ("32x0e+16x0e+32x1o", "32x0e+32x1o+8x2e", True, 70),
]


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def main():
    import oracle.o3 as oo3
    from gnn.o3 import Linear
    bad = 0
    for irin, irout, bias, n in CASES:
        torch.manual_seed(3)
        o = oo3.Linear(irin, irout, biases=bias).double()
        m = Linear(irin, irout, biases=bias).to("cuda")
        with torch.no_grad():
            if bias:
                o.bias.normal_()
            for k, p in m.named_parameters():
                p.copy_(dict(o.named_parameters())[k].float())
        x = torch.randn(n, o.irreps_in.dim, dtype=torch.float64)
        xo = x.clone().requires_grad_(True)
        yo = o(xo)
        g = torch.randn_like(yo)
        (yo * g).sum().backward()
        xm = x.float().cuda().requires_grad_(True)
        ym = m(xm)
        (ym * g.float().cuda()).sum().backward()
        e = [rel(ym, yo), rel(xm.grad, xo.grad), rel(m.weight.grad, o.weight.grad)]
        ok = e[0] < 2e-6 and e[1] < 2e-6 and e[2] < 5e-6
        if not ok:
            bad += 1
            # which weight block is off
            wm, wo = m.weight.grad.double().cpu(), o.weight.grad
            for (i, oo), off in zip(m.instructions, m._w_offs):
                k = m.irreps_in[i].mul * m.irreps_out[oo].mul
                eb = rel(wm[off:off + k], wo[off:off + k])
                if eb > 5e-6:
                    print(f"     grad-W block ins ({i},{oo}) {m.irreps_in[i]}->{m.irreps_out[oo]} rel {eb:.2e}")
            yd = (ym.detach().double().cpu() - yo.detach()).abs().max(0).values
            cols = torch.nonzero(yd > 1e-5 * yo.abs().max()).flatten().tolist()
            if cols:
                print(f"     fwd bad columns {cols[:8]}... ({len(cols)}) rows "
                      f"{torch.nonzero((ym.detach().double().cpu() - yo.detach()).abs().max(1).values > 1e-5 * yo.abs().max()).flatten().tolist()[:10]}")
        print(f"{'ok ' if ok else 'BAD'} {irin[:30]:30s} -> {irout[:30]:30s} n={n:5d} "
              f"fwd {e[0]:.1e} gx {e[1]:.1e} gw {e[2]:.1e}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
