"""Fused radial MLP (csrc/eelg_radial.hip, C ABI eelg_radial_fwd / eelg_radial_bwd) against a
float64 PyTorch restatement of the reference's ``conv_tp_weights`` Sequential
(gnn/blocks.py:537-549): Linear(F, H) + SiLU, (Linear(H, H) + SiLU) * (layers - 2),
Linear(H, W, bias=False).

Tolerances (fp32 MFMA vs fp64), stated per test: forward output and every weight / bias
gradient within 1e-5 * max|ref| (fp32 storage); bf16 storage of the output and of its
gradient: 1e-2 * max|ref| on the output (bf16 rounding, 2^-8 relative) and 2e-5 on the
weight gradients given the same bf16 grad_w input.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return round(float((a - b).abs().max() / b.abs().max().clamp_min(1e-30)), 9)


def _mlp(n_feat, hidden, layers, n_out, seed):
    torch.manual_seed(seed)
    last = torch.nn.Linear(hidden, n_out, bias=False)
    torch.nn.init.xavier_uniform_(last.weight, gain=10)
    seq = torch.nn.Sequential(torch.nn.Linear(n_feat, hidden), torch.nn.SiLU())
    for _ in range(layers - 2):
        seq.append(torch.nn.Linear(hidden, hidden))
        seq.append(torch.nn.SiLU())
    seq.append(last)
    return seq


@pytest.mark.parametrize("n_edges,n_feat,hidden,layers,n_out", [
    (4096, 12, 64, 3, 1344),     # config 2, layers >= 1
    (1000, 12, 64, 3, 160),      # config 2, layer 0 (ragged edge count)
    (77, 12, 64, 3, 736),        # config 5 width, fewer edges than one workgroup
    (513, 7, 32, 2, 100),        # odd feature count, one hidden layer, ragged width
    (300, 12, 64, 4, 50),        # three hidden layers
    (1, 12, 32, 4, 33),          # a single edge
])
def test_radial_mlp_fwd_bwd_fp32(n_edges, n_feat, hidden, layers, n_out):
    from gnn import ops
    ref = _mlp(n_feat, hidden, layers, n_out, seed=n_edges).double()
    dev = _mlp(n_feat, hidden, layers, n_out, seed=n_edges).to(DEV)
    torch.manual_seed(1)
    feats = torch.rand(n_edges, n_feat, dtype=torch.float64) * 0.9
    g = torch.randn(n_edges, n_out, dtype=torch.float64)
    yr = ref(feats)
    (yr * g).sum().backward()
    yd = ops.radial_mlp(feats.float().to(DEV), dev)
    (yd * g.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert yd.dtype == torch.float32 and yd.shape == (n_edges, n_out)
    assert rel_err(yd, yr) < 1e-5
    pr = dict(ref.named_parameters())
    for name, p in dev.named_parameters():
        assert rel_err(p.grad, pr[name].grad) < 1e-5, name


def test_radial_mlp_bf16_storage():
    from gnn import ops
    n_edges, n_out = 2000, 736
    ref = _mlp(12, 64, 3, n_out, seed=5).double()
    dev = _mlp(12, 64, 3, n_out, seed=5).to(DEV)
    torch.manual_seed(2)
    feats = torch.rand(n_edges, 12, dtype=torch.float64) * 0.9
    g = torch.randn(n_edges, n_out).to(torch.bfloat16)
    yr = ref(feats)
    (yr * g.double()).sum().backward()          # the bf16 gradient, widened exactly
    yd = ops.radial_mlp(feats.float().to(DEV), dev, torch.bfloat16)
    assert yd.dtype == torch.bfloat16
    yd.backward(g.to(DEV))
    torch.cuda.synchronize()
    assert rel_err(yd.float(), yr) < 1e-2
    pr = dict(ref.named_parameters())
    for name, p in dev.named_parameters():
        assert rel_err(p.grad, pr[name].grad) < 2e-5, name


def test_radial_mlp_zero_edges():
    from gnn import ops
    dev = _mlp(12, 64, 3, 1344, seed=0).to(DEV)
    feats = torch.zeros(0, 12, device=DEV)
    y = ops.radial_mlp(feats, dev)
    assert y.shape == (0, 1344)
    y.sum().backward()
    for p in dev.parameters():
        assert p.grad is not None and float(p.grad.abs().max()) == 0.0


def test_radial_mlp_deterministic():
    """Two runs give bit-identical outputs and gradients (no atomics anywhere)."""
    from gnn import ops
    dev = _mlp(12, 64, 3, 1344, seed=3).to(DEV)
    feats = torch.rand(10000, 12, device=DEV)
    g = torch.randn(10000, 1344, device=DEV)
    outs = []
    for _ in range(2):
        dev.zero_grad()
        y = ops.radial_mlp(feats, dev)
        y.backward(g)
        outs.append([y.detach().clone()] + [p.grad.clone() for p in dev.parameters()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_split_bf16x3_is_exact():
    """``eelg_split_bf16x3``: three bf16 parts whose sum is the fp32 input bit for bit (normal
    range, both signs, zeros), the operand form of the fp32-accurate bf16 MFMA GEMMs."""
    from gnn import ops
    torch.manual_seed(3)
    x = torch.randn(100003, device=DEV) * torch.logspace(-20, 20, 100003, device=DEV)
    x[:7] = torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0000002, 1e-30, -7.1e20], device=DEV)
    p = ops.split_bf16x3(x)
    assert p.dtype == torch.bfloat16 and p.shape == (3,) + x.shape
    back = (p[0].float() + p[1].float()) + p[2].float()      # each partial sum is exact
    assert torch.equal(back, x)


@pytest.mark.parametrize("hidden,n_out", [(64, 1344), (32, 160)])
def test_radial_split_gemm_as_accurate_as_fp32(hidden, n_out):
    """The output layer and its gradients run on bf16 MFMA with split operands (six part
    products, fp32 accumulation).  Against fp64, their error must be that of fp32 arithmetic:
    at most 1.5x the error of the same MLP evaluated by torch in fp32 on the device (plus
    1e-7 of the output scale), forward and every weight gradient."""
    from gnn import ops
    n_edges = 8192
    ref = _mlp(12, hidden, 3, n_out, seed=11).double()
    dev = _mlp(12, hidden, 3, n_out, seed=11).to(DEV)
    f32 = _mlp(12, hidden, 3, n_out, seed=11).to(DEV)
    torch.manual_seed(2)
    feats = torch.rand(n_edges, 12, dtype=torch.float64) * 0.9
    g = torch.randn(n_edges, n_out, dtype=torch.float64)
    yr = ref(feats)
    (yr * g).sum().backward()
    yd = ops.radial_mlp(feats.float().to(DEV), dev)
    (yd * g.float().to(DEV)).sum().backward()
    yf = f32(feats.float().to(DEV))
    (yf * g.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    e_split, e_f32 = rel_err(yd, yr), rel_err(yf, yr)
    assert e_split <= 1.5 * e_f32 + 1e-7, (e_split, e_f32)
    pr, pf = dict(ref.named_parameters()), dict(f32.named_parameters())
    errs = {name: (rel_err(p.grad, pr[name].grad), rel_err(pf[name].grad, pr[name].grad))
            for name, p in dev.named_parameters()}
    print("rel err vs fp64 (device, torch fp32):", errs)   # shown on failure
    for name, (es, ef) in errs.items():
        assert es <= 1.5 * ef + 1e-7, (name, es, ef)


@pytest.mark.parametrize("n_edges,layers,bf16", [(4096, 3, False), (1000, 2, False), (77, 4, False),
                                                 (4096, 3, True)])
def test_radial_chain_backward_matches_fused_backward(n_edges, layers, bf16, monkeypatch):
    """hidden 64: the chain backward (``eelg_radial_bwd_chain`` + weight gradients on the linear
    weight-gradient kernel + column sums) against the fused small-layer kernel
    (``eelg_radial_bwd``), same inputs: the output-weight gradient bitwise (same kernel), the
    hidden-layer gradients within 2e-6 of their max (another fp32 summation order)."""
    from gnn import ops
    dev = _mlp(12, 64, layers, 1344, seed=5).to(DEV)
    torch.manual_seed(2)
    feats = (torch.rand(n_edges, 12) * 0.9).to(DEV)
    g = torch.randn(n_edges, 1344, device=DEV)
    dt = torch.bfloat16 if bf16 else torch.float32

    def grads(chain):
        monkeypatch.setattr(ops, "RADIAL_CHAIN", chain)
        for p in dev.parameters():
            p.grad = None
        y = ops.radial_mlp(feats, dev, out_dtype=dt)
        y.backward(g.to(dt))
        return [p.grad.clone() for p in dev.parameters()]
    a, b = grads(True), grads(False)
    for k, (u, v) in enumerate(zip(a, b)):
        if k == len(a) - 1:
            assert torch.equal(u, v)
        else:
            assert rel_err(u, v) < 2e-6, k
