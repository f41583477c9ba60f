"""CGC / mCGC benchmark models: oracle checks on CPU, HIP parity
on the GPU (fp32 HIP vs fp64 oracle; layer 2e-5, model 1e-4 relative to max, grads 2e-5)."""
from argparse import Namespace

import pytest
import torch

import oracle.cgc as ocgc
from helpers import batch, batch_to

F64 = torch.float64


def cgc_params(hidden=32, reduction="sum", positive="square", passes=3):
    return Namespace(hidden_irreps=hidden, interaction_reduction=reduction, global_reduction="mean",
                     message_passes=passes, positive=positive)


def test_oracle_cgc_layer_formula():
    """msg_e = softplus(W_v c + b_v) * sigmoid(W_m c + b_m), summed at the receiver."""
    torch.manual_seed(0)
    layer = ocgc.CGCLayer(4, 4).double()
    x = torch.randn(3, 4, dtype=F64)
    ef = torch.randn(2, 4, dtype=F64)
    ei = torch.tensor([[0, 2], [1, 1]])
    out = layer(x, ei, ef)
    manual = torch.zeros(3, 4, dtype=F64)
    for e in range(2):
        c = torch.cat([x[ei[0, e]], x[ei[1, e]], ef[e]])
        v = layer.fc_values.weight @ c + layer.fc_values.bias
        m = layer.fc_multip.weight @ c + layer.fc_multip.bias
        manual[ei[1, e]] += torch.log1p(torch.exp(v)) / (1 + torch.exp(-m))
    assert torch.allclose(out, manual, atol=1e-12)


def test_oracle_mcgc_output_symmetric_psd_and_param_count():
    torch.manual_seed(0)
    m = ocgc.CrystGraphConv(cgc_params(hidden=128)).double()
    # reference params (scripts/train_cgcnn_modified.py:26-30): 324,245 weights
    assert sum(p.numel() for p in m.parameters()) == 324245
    b, _ = batch(2, 20, 80, 5)
    c = m(batch_to(b, "cpu", F64))["stiffness"]
    assert torch.allclose(c, c.transpose(1, 2))
    assert (torch.linalg.eigvalsh(c) > -1e-10).all()


def test_product_cgc_param_names_match_oracle():
    from gnn.cgc import CrystGraphConv, CrystGraphConvVanilla
    for pc, oc in ((CrystGraphConv, ocgc.CrystGraphConv), (CrystGraphConvVanilla, ocgc.CrystGraphConvVanilla)):
        a, o = pc(cgc_params(64)), oc(cgc_params(64))
        assert {k: v.shape for k, v in a.named_parameters()} == {k: v.shape for k, v in o.named_parameters()}


def test_benchmark_models_import_path():
    from benchmark_models.cgc_modified import CrystGraphConv as A
    from benchmark_models.cgc_vanilla import CrystGraphConv as B
    from gnn.cgc import CrystGraphConv, CrystGraphConvVanilla
    assert A is CrystGraphConv and B is CrystGraphConvVanilla


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("reduction,d", [("sum", 128), ("mean", 64), ("sum", 96), ("sum", 192),
                                         ("mean", 256)])
def test_cgc_layer_fwd_bwd(reduction, d):
    """One CGC layer against the fp64 oracle, every node width class of the kernels: D <= 64
    (1 float per lane), <= 128 (2) and <= 256 (4 floats per lane, CGC_MAXD)."""
    from gnn.cgc import CGCLayer
    torch.manual_seed(1)
    o = ocgc.CGCLayer(d, d, reduction).double()
    m = CGCLayer(d, d, reduction).cuda()
    m.load_state_dict({k: v.float() for k, v in o.state_dict().items()})
    b, _ = batch(3, 40, 160, 11)
    ei = b.edge_index
    n, e = b.node_attrs.shape[0], ei.shape[1]
    x = torch.randn(n, d, dtype=F64)
    ef = torch.randn(e, d, dtype=F64)
    ei[:, 5] = ei[:, 4]                      # a repeated edge
    xo, eo = x.clone().requires_grad_(True), ef.clone().requires_grad_(True)
    yo = o(xo, ei, eo)
    g = torch.randn_like(yo)
    (yo * g).sum().backward()
    xm, em = x.float().cuda().requires_grad_(True), ef.float().cuda().requires_grad_(True)
    ym = m(xm, ei.cuda(), em)
    (ym * g.float().cuda()).sum().backward()
    assert _rel(ym, yo) < 2e-5
    assert _rel(xm.grad, xo.grad) < 2e-5
    assert _rel(em.grad, eo.grad) < 2e-5
    po = dict(o.named_parameters())
    for k, p in m.named_parameters():
        assert _rel(p.grad, po[k].grad) < 2e-5, k


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["modified", "vanilla"])
def test_cgc_model_fwd_bwd_matches_oracle(variant):
    from gnn import cgc
    torch.manual_seed(0)
    p = cgc_params(hidden=128 if variant == "modified" else 64)
    oc, pc = ((ocgc.CrystGraphConv, cgc.CrystGraphConv) if variant == "modified"
              else (ocgc.CrystGraphConvVanilla, cgc.CrystGraphConvVanilla))
    o = oc(p).double()
    m = pc(p).cuda()
    m.load_state_dict({k: v.float() for k, v in o.state_dict().items()})
    b, _ = batch(4, 50, 200, 1234)
    co = o(batch_to(b, "cpu", F64))["stiffness"]
    t = torch.randn_like(co)
    (co * t).sum().backward()
    cm = m(b.to("cuda"))["stiffness"]
    (cm * t.float().cuda()).sum().backward()
    assert _rel(cm, co) < 1e-4
    po = dict(o.named_parameters())
    # every parameter gradient within 2e-5 of its own largest entry (fp32 vs fp64)
    for k, q in m.named_parameters():
        assert _rel(q.grad, po[k].grad) < 2e-5, k


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["modified", "vanilla"])
def test_cgc_model_fullsize_matches_oracle(variant):
    """BASELINE config 4 at the bench shape per graph (1024 nodes / 4096 edges, 2 graphs):
    stiffness 1e-4, every parameter gradient 2e-5 of its largest entry."""
    from gnn import cgc
    torch.manual_seed(1)
    p = cgc_params(hidden=128 if variant == "modified" else 64)
    oc, pc = ((ocgc.CrystGraphConv, cgc.CrystGraphConv) if variant == "modified"
              else (ocgc.CrystGraphConvVanilla, cgc.CrystGraphConvVanilla))
    o = oc(p).double()
    m = pc(p).cuda()
    m.load_state_dict({k: v.float() for k, v in o.state_dict().items()})
    b, _ = batch(2, 1024, 4096, 4321)
    co = o(batch_to(b, "cpu", F64))["stiffness"]
    t = torch.randn_like(co)
    (co * t).sum().backward()
    cm = m(b.to("cuda"))["stiffness"]
    (cm * t.float().cuda()).sum().backward()
    po = dict(o.named_parameters())
    worst = max(_rel(q.grad, po[k].grad) for k, q in m.named_parameters())
    from helpers import record_parity
    record_parity(f"cgc_{variant}_fullsize", stiffness=_rel(cm, co), grad_params=worst)
    assert _rel(cm, co) < 1e-4
    for k, q in m.named_parameters():
        assert _rel(q.grad, po[k].grad) < 2e-5, k


@pytest.mark.gpu
@pytest.mark.parametrize("k,n_out,bias,rows", [(128, 256, True, 1000), (96, 192, False, 1000),
                                               (64, 21, True, 1000), (32, 64, True, 1000),
                                               (5, 128, True, 1000), (128, 256, True, 6000),
                                               (96, 192, False, 4100), (64, 21, True, 5000),
                                               (32, 300, True, 4096)])
def test_dense_linear_matches_torch(k, n_out, bias, rows):
    """``gnn.dense.Linear`` (the CGC models' Linear layers on the in-tree MFMA kernels): output,
    grad-x, grad-W and grad-b against the fp64 torch Linear, 2e-6 of the largest entry (fp32
    sums over K / over the rows).  K >= 128 forward / grad-x and, from 4096 rows, the weight
    gradient run on the split-bf16 kernels (ragged last row tile and output blocks included)."""
    from gnn import dense
    torch.manual_seed(3)
    ref = torch.nn.Linear(k, n_out, bias=bias).double()
    m = dense.Linear(k, n_out, bias=bias).cuda()
    m.load_state_dict({kk: v.float() for kk, v in ref.state_dict().items()})
    x = torch.randn(rows, k, dtype=F64)
    xo, xm = x.clone().requires_grad_(True), x.float().cuda().requires_grad_(True)
    yo, ym = ref(xo), m(xm)
    g = torch.randn_like(yo)
    (yo * g).sum().backward()
    (ym * g.float().cuda()).sum().backward()
    assert _rel(ym, yo) < 2e-6
    assert _rel(xm.grad, xo.grad) < 2e-6
    assert _rel(m.weight.grad, ref.weight.grad) < 2e-6
    if bias:
        assert _rel(m.bias.grad, ref.bias.grad) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("d", [128, 192, 256])
def test_cgc_factored_edges_match_generic_layer(d):
    """``CGCLayer.forward_factored`` (edge features as [e5 | 1] @ A, eelg_cgc_fwd_ef) equals the
    generic ``forward`` on the materialised edge features e5 W5^T + b5 (two fp32 evaluations in
    different association orders: 1e-5 of the largest entry), gradients w.r.t. x and the layer
    weights included, and the edge embedding's gradients agree."""
    from gnn import cgc
    from gnn.model import EnergyEquivGNN
    torch.manual_seed(4)
    layer = cgc.CGCLayer(d, d).cuda()
    emb = torch.nn.Linear(5, d).cuda()
    b, _ = batch(3, 40, 160, 17)
    bd = b.to("cuda")
    csr = EnergyEquivGNN.edge_graph(bd)
    e5 = cgc._edge_inputs(bd, csr)
    ef = torch.cat([e5, torch.ones_like(e5[:, :1]), torch.zeros_like(e5[:, :2])], 1).contiguous()
    x = torch.randn(csr.num_nodes, d, device="cuda")
    g = torch.randn(csr.num_nodes, d, device="cuda")

    def run(factored):
        for p in list(layer.parameters()) + list(emb.parameters()):
            p.grad = None
        xr = x.clone().requires_grad_(True)
        if factored:
            y = layer.forward_factored(xr, csr, ef, cgc._edge_factor(emb, layer.edge_block()))
        else:
            y = layer(xr, csr, emb(e5))
        (y * g).sum().backward()
        return [y.detach(), xr.grad] + [p.grad.clone() for p in list(layer.parameters()) + list(emb.parameters())]
    a, r = run(True), run(False)
    for u, v in zip(a, r):
        assert _rel(u, v) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("d,reduction", [(128, "sum"), (64, "mean"), (192, "sum"), (256, "mean")])
def test_cgc_fused_residual_matches_explicit_add(d, reduction):
    """``forward_factored(..., residual=True)`` (x + layer(x) with the add in the aggregation
    kernel's store and its gradient in grad-x's epilogue) equals the explicit ``x + layer(x)``:
    output bitwise (one fp32 add either way), gradients within 1e-6 of their largest entry."""
    from gnn import cgc
    from gnn.model import EnergyEquivGNN
    torch.manual_seed(5)
    layer = cgc.CGCLayer(d, d, reduction).cuda()
    emb = torch.nn.Linear(5, d).cuda()
    b, _ = batch(3, 40, 160, 17)
    bd = b.to("cuda")
    csr = EnergyEquivGNN.edge_graph(bd)
    e5 = cgc._edge_inputs(bd, csr)
    ef = torch.cat([e5, torch.ones_like(e5[:, :1]), torch.zeros_like(e5[:, :2])], 1).contiguous()
    x = torch.randn(csr.num_nodes, d, device="cuda")
    g = torch.randn(csr.num_nodes, d, device="cuda")

    def run(fused):
        for p in list(layer.parameters()) + list(emb.parameters()):
            p.grad = None
        xr = x.clone().requires_grad_(True)
        ea = cgc._edge_factor(emb, layer.edge_block())
        y = layer.forward_factored(xr, csr, ef, ea, residual=True) if fused else \
            xr + layer.forward_factored(xr, csr, ef, ea)
        (y * g).sum().backward()
        return [y.detach(), xr.grad] + [p.grad.clone() for p in list(layer.parameters()) + list(emb.parameters())]
    a, r = run(True), run(False)
    assert torch.equal(a[0], r[0])
    for u, v in zip(a[1:], r[1:]):
        assert _rel(u, v) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("k,n_out,bias,rows", [(1, 128, True, 5000), (3, 64, True, 777), (3, 32, False, 300)])
def test_small_in_linear_matches_fp64(k, n_out, bias, rows):
    """The node embeddings' K <= 8 linear (dense.small_in_linear: addcmul forward, weight and bias
    gradients as sum_rows column sums) against an fp64 torch linear: output, weight and bias
    gradients within 2e-6 of their largest entry."""
    from gnn import dense
    torch.manual_seed(0)
    lin = dense.SmallInLinear(k, n_out, bias=bias).cuda()
    x = torch.randn(rows, k, device="cuda")
    g = torch.randn(rows, n_out, device="cuda")
    y = lin(x)
    y.backward(g)
    w64 = lin.weight.detach().double().requires_grad_(True)
    b64 = lin.bias.detach().double().requires_grad_(True) if bias else None
    y64 = torch.nn.functional.linear(x.double(), w64, b64)
    y64.backward(g.double())

    def rel(a, b):
        return float((a.detach().double() - b.detach()).abs().max() / b.detach().abs().max())
    assert rel(y, y64) < 2e-6
    assert rel(lin.weight.grad, w64.grad) < 2e-6
    if bias:
        assert rel(lin.bias.grad, b64.grad) < 2e-6


@pytest.mark.gpu
def test_cgc_softplus_sigmoid_match_torch_over_the_range():
    """The kernels' fast-math softplus and sigmoid (hardware exp2 / log2 / rcp, CGC_FAST_MATH)
    against torch's fp64 softplus (threshold 20) and sigmoid over z in [-30, 20], through the
    C-ABI forward: one self-edge per receiver, ps = ep = 0, pr = [zv | zm], so
    agg = softplus(zv) * sigmoid(zm).  With zm = 40 (sigmoid = 1.0f) agg is softplus alone,
    relative error <= 5e-6 everywhere, including z < -16.6 where softplus ~ exp(z) (the bound is
    the fp32 rounding of the exp2 argument, |z| log2(e) 2^-24 ln 2 = 1.8e-6 at z = -30); with
    zv = 30 (softplus = z) agg is 30 * sigmoid(zm)."""
    from gnn import _lib
    lib = _lib.load()
    d = 64
    z = torch.linspace(-30.0, 20.0, 4096 * d, dtype=F64).reshape(-1, d)
    n = z.shape[0]
    rowptr = torch.arange(n + 1, dtype=torch.int32, device="cuda")
    sender = torch.arange(n, dtype=torch.int32, device="cuda")
    ps = torch.zeros(n, 2 * d, device="cuda")
    ep = torch.zeros(n, 2 * d, device="cuda")
    for which in ("softplus", "sigmoid"):
        zf = z.float()
        fixed = torch.full_like(zf, 40.0 if which == "softplus" else 30.0)
        pr = (torch.cat([zf, fixed], 1) if which == "softplus" else torch.cat([fixed, zf], 1)).cuda().contiguous()
        agg = torch.empty(n, d, device="cuda")
        _lib.check(lib.eelg_cgc_fwd(_lib.ptr(ps), _lib.ptr(pr), _lib.ptr(ep), _lib.ptr(sender),
                                    _lib.ptr(rowptr), None, n, d, _lib.ptr(agg), _lib.stream(agg)), "cgc_fwd")
        zr = zf.double()
        ref = (torch.nn.functional.softplus(zr) if which == "softplus" else 30.0 * torch.sigmoid(zr))
        rel = ((agg.double().cpu() - ref).abs() / ref.abs()).max().item()
        assert rel < 5e-6, (which, rel)
