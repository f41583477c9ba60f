#!/usr/bin/env python3
"""Benchmark: lattice-graphs/s (fwd+bwd) of the 4-layer EnergyEquivGNN training step.

Workload (BASELINE.json configs[1]; configs[2] at 8 GPUs): synthetic periodic
lattices of 1024 nodes / 4096 directed edges, 32 graphs per GPU per step,
4 message passes, the reference's network params (``scripts/train_main.py:25-52``).
One step = forward + relative-MSE loss + backward + flat fp32 gradient
all-reduce (N>1, RCCL) + grad-norm clip 10 + AdamW(amsgrad) step.  Graphs are
sharded by graph id across ranks (weak scaling); inputs are resident in HBM
before the timed region.

Run: ``python bench.py [--gpus N --steps K --warmup W]``.  For N > 1 the driver uses
``torch.distributed.run`` and each rank reads RANK/LOCAL_RANK/WORLD_SIZE; without a
launcher ``--gpus N`` starts the N rank processes itself (``launch_ranks``).
Rank 0 prints one JSON line (roofline of the fused interaction kernel measured
with HIP events over the timed region; CPU baseline = the oracle restatement).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "energy-equiv-lattice-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FETCH_CORRECTION = 2.0   # HBM read bytes per FETCH_SIZE byte on gfx950 (measured, any load width)


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _spawned_rank(local_rank: int, world: int, port: int, argv):
    """Entry point of a rank started by ``launch_ranks`` (a fresh interpreter: spawn)."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def launch_ranks(n: int) -> None:
    """``bench.py --gpus N`` without a launcher: start N rank processes (spawn, i.e. fresh
    interpreters, before this process touches the GPU) and wait for them; they read
    RANK/LOCAL_RANK/WORLD_SIZE like ranks under ``torch.distributed.run``."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned_rank, args=(n, _free_port(), sys.argv[1:]), nprocs=n, join=True,
                       start_method="spawn")


def init_dist(rehearsal: bool = False):
    """(world, rank, local_rank, device, n_devices, backend) of this rank.  One process per GPU
    over RCCL (backend 'nccl').  With fewer visible devices than ranks the ranks would have to
    share devices over gloo: that is only a rehearsal of the multi-rank code path, not a
    multi-GPU measurement, so it is refused unless ``--rehearsal`` is given (and the JSON line
    then names the backend and says so)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    backend = None
    if world > 1:
        if ndev >= world:
            backend = "nccl"
        elif rehearsal:
            backend = "gloo"
        else:
            raise SystemExit(f"bench.py: {world} ranks but {ndev} visible GPU(s): refusing to report a "
                             f"dp{world} number over gloo on shared devices (pass --rehearsal to run "
                             "the multi-rank path anyway, labelled as a rehearsal)")
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    elif backend == "gloo":
        dist.init_process_group("gloo")
    return world, rank, local_rank, dev, min(world, ndev), backend


def params_equal_across_ranks(params) -> bool:
    """Bitwise equality of every parameter across ranks (elementwise max == min all-reduce)."""
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    hi, lo = flat.clone(), flat.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))


def make_params(layers: int, max_edge_radius: float, lmax: int = 4, storage: str = "float32",
                correlation: int = 3):
    from argparse import Namespace
    hid = "+".join(f"32x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    ro = "+".join(f"16x{l}{'e' if l % 2 == 0 else 'o'}" for l in range(lmax + 1))
    return Namespace(lmax=lmax, hidden_irreps=hid, readout_irreps=ro, num_edge_bases=6,
                     interaction_reduction="sum", interaction_bias=True, agg_norm_const=4.0,
                     inter_MLP_dim=64, inter_MLP_layers=3, correlation=correlation, global_reduction="mean",
                     message_passes=layers, positive_function="matrix_power_2",
                     max_edge_radius=max_edge_radius, lr=1e-3, beta1=0.9, epsilon=1e-8,
                     amsgrad=True, weight_decay=1e-8, storage_dtype=storage)


def tp_fwd_bytes(n: int, e: int, din: int, w: int, dmid: int, nsh: int = 25, wbytes: int = 4) -> int:
    """Algorithmic bytes of one fused-interaction launch ('Fused TP+scatter'):
    x[N,Din] + sh[E,nsh] + w[E,W] + sender[E] + rowptr[N+1] (read) + agg[N,Dmid] (write);
    w is ``wbytes`` per element (2 with bf16 storage, BASELINE config 5)."""
    return 4 * (n * din + e * nsh + e + (n + 1) + n * dmid) + wbytes * e * w


def workload_key(args) -> str:
    """Key of this command's workload in profiles/pmc_traffic.json (tools/summarize_profile.py)."""
    if args.model != "egnn":
        return f"{args.model}_b{args.batch}_n{args.nodes}_e{args.edges}"
    return (f"egnn_b{args.batch}_n{args.nodes}_e{args.edges}_L{args.layers}_lmax{args.lmax}_"
            f"{args.storage}")


def pmc_traffic(kernel: str, args) -> dict | None:
    """HBM bytes per launch of ``kernel`` from the committed PMC table (profiles/pmc_traffic.json,
    written by tools/summarize_profile.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    of this same command: tools/profile_round.sh with BENCH_ARGS), looked up under this
    command's workload key; None when that workload has no committed passes."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    tab = json.load(open(path)).get("workloads", {}).get(workload_key(args))
    if tab is None:
        return None
    def base(name):   # "void cgc_fwd_kernel<2>" -> "cgc_fwd_kernel"
        name = name.split("|")[0]
        name = name[5:] if name.startswith("void ") else name
        return name.split("<")[0]
    hits = [v for k, v in tab["kernels"].items() if base(k) == kernel]
    if not hits:
        return None
    t = max(hits, key=lambda v: sum(v.values()))
    fetch_raw, write = t.get("FETCH_SIZE", 0.0), t.get("WRITE_SIZE", 0.0)
    # gfx950 calibration (profiles/r02_fetch_calibration.md, tools/proto/fetch_calib.hip): a
    # kernel reading 1 GiB once reports FETCH_SIZE = 0.500 GiB at 4, 8, 12 and 16 B per lane;
    # WRITE_SIZE reports 1.000 GiB for 1 GiB written.  HBM read bytes = 2 x FETCH_SIZE.
    fetch = FETCH_CORRECTION * fetch_raw
    return {"bytes": round(fetch + write), "fetch": round(fetch), "write": round(write),
            "fetch_raw": round(fetch_raw), "fetch_correction": FETCH_CORRECTION,
            "source": f"profiles/pmc_traffic.json [{workload_key(args)}] ({tab['source']}), "
                      "calibration profiles/r02_fetch_calibration.md"}


def host_cpu() -> dict:
    """The host cores this process may use: the cgroup CPU quota when one is set (the GPU box
    gives each job a share of a larger machine), else the affinity mask; plus the CPU model."""
    n_aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": min(n_aff, quota) if quota else n_aff, "os_cpu_count": os.cpu_count(),
            "affinity": n_aff, "cgroup_quota": quota, "model": model,
            "isa": torch.backends.cpu.get_cpu_capability()}


def _time_cpu_steps(step, budget_s: float, warmup: int, min_steps: int, max_steps: int,
                    progress: str = ""):
    """``warmup`` untimed steps, then timed steps until ``min_steps`` are done and the budget is
    spent, or ``max_steps`` are done (3 warm-up + >= 10 timed).
    ``progress``: a label; one line per step goes to stderr (a long CPU leg is not silent)."""
    for i in range(warmup):
        t0 = time.perf_counter()
        step()
        if progress:
            print(f"{progress}: warm-up {i + 1}/{warmup} {time.perf_counter() - t0:.2f} s",
                  file=sys.stderr, flush=True)
    times, t_start = [], time.perf_counter()
    while len(times) < max_steps:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        if progress:
            print(f"{progress}: timed {len(times)} {times[-1]:.2f} s", file=sys.stderr, flush=True)
        if len(times) >= min_steps and time.perf_counter() - t_start > budget_s:
            break
    times.sort()
    return times


def cpu_baseline(n_nodes: int, n_edges: int, layers: int, budget_s: float, lmax: int = 4,
                 full: bool = True, correlation: int = 3):
    """The oracle (pure-PyTorch CPU restatement of the reference, dense per-path TP,
    scatter_add_, opt_einsum-order symmetric contraction) on ONE graph of the same
    shape: fwd + loss + bwd on all the host cores this job has.  ``full`` (default):
    BASELINE.md section 2's protocol, 3 warm-up + 10 timed steps (about 3.5 min on 16 EPYC
    threads); ``full=False`` (``bench.py --cpu-quick``): 1 warm-up and timed steps within
    ``budget_s`` (at least 1)."""
    import oracle.model as om
    from oracle.train import stiffness_loss
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    host = host_cpu()
    torch.set_num_threads(host["threads"])
    ds = SyntheticLattices(1, n_nodes, n_edges, 1234)
    b = collate([ds[0]])
    torch.manual_seed(0)
    m = om.EnergyEquivGNN(make_params(layers, ds.max_edge_radius, lmax, correlation=correlation))

    def step():
        m.zero_grad(set_to_none=True)
        stiffness_loss(m(b)["stiffness"], b.stiffness).backward()

    warm, lo, hi = (3, 10, 10) if full else (1, 1, 10)
    t = _time_cpu_steps(step, budget_s, warm, lo, hi, progress="cpu_baseline")
    med = statistics.median(t)
    pct = lambda q: t[min(len(t) - 1, int(q * (len(t) - 1) + 0.5))]  # noqa: E731
    return {"value": round(1.0 / med, 4), "unit": "lattice-graphs/s", "cores": host["threads"],
            "kind": "port", "cpu": host,
            "sample": f"oracle fp32 fwd+loss+bwd, 1 graph x {n_nodes} nodes/{n_edges} edges, "
                      f"{layers} layers lmax {lmax}; {warm} warm-up + {len(t)} timed step(s): median "
                      f"{med:.2f} s, p10 {pct(0.1):.2f} s, p90 {pct(0.9):.2f} s" +
                      (" (BASELINE.md section 2 protocol)" if full else
                       f" (budget {budget_s:.0f} s, bench.py --cpu-quick; BASELINE.md section 2's "
                       "3 + 10 steps are the default)")}


def inline_kernel_times(step, steps: int) -> dict:
    """Per-op HIP-event times (ops.TIMER) over ``steps`` training steps run in line: every kernel
    on the main stream in EELG_OVERLAP=0's order (one untimed step first).  The side-stream overlap
    is switched back on afterwards.  Every rank runs it (the step holds the all-reduce)."""
    from gnn import ops
    saved = ops.OVERLAP
    ops.OVERLAP = False
    try:
        step()
        torch.cuda.synchronize()
        ops.TIMER.enabled = True
        ops.TIMER.records.clear()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ops.TIMER.enabled = False
        return ops.TIMER.summary()
    finally:
        ops.TIMER.enabled = False
        ops.OVERLAP = saved


def cgc_fwd_bytes(n: int, e: int, d: int, residual: bool = False) -> int:
    """Algorithmic bytes of one fused CGC edge-conv launch on factored edge features
    (``eelg_cgc_fwd_ef``, the models' path): node projections ps, pr [N, 2D] read once, the
    8-float edge rows ef [E, 8] and A [8, 2D], sender [E] + rowptr [N+1], agg [N, D] written;
    with the layer residual (``eelg_cgc_fwd_ef_res``) the layer input h [N, D] is read too."""
    return 4 * (2 * n * 2 * d + e * 8 + 8 * 2 * d + e + (n + 1) + n * d + (n * d if residual else 0))


def cpu_baseline_cgc(modified: bool, p, n_nodes: int, n_edges: int, budget_s: float):
    """The CGC oracle (oracle/cgc.py, the reference's torch ops on CPU) on one graph of the
    same shape: fwd + loss + bwd, median over steps within ``budget_s``."""
    import oracle.cgc as ocgc
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    ds = SyntheticLattices(1, n_nodes, n_edges, 1234)
    b = collate([ds[0]])
    torch.manual_seed(0)
    m = (ocgc.CrystGraphConv if modified else ocgc.CrystGraphConvVanilla)(p)
    iu = torch.triu_indices(6, 6)
    tgt = b.stiffness if modified else b.stiffness[:, iu[0], iu[1]]
    host = host_cpu()
    torch.set_num_threads(host["threads"])

    def step():
        m.zero_grad(set_to_none=True)
        stiffness_loss(m(b)["stiffness"], tgt).backward()

    times = _time_cpu_steps(step, budget_s, 3, 10, 50)
    med = statistics.median(times)
    return {"value": round(1.0 / med, 3), "unit": "lattice-graphs/s", "cores": host["threads"],
            "kind": "port", "cpu": host,
            "sample": f"oracle fp32 fwd+loss+bwd, 1 graph x {n_nodes} nodes/{n_edges} "
                      f"edges, 3 warm-up + median of {len(times)} step(s) ({med * 1e3:.1f} ms/step)"}


def main_cgc(args):
    """BASELINE config 4: CGC / mCGC (scripts/train_cgcnn_*.py) on the same synthetic lattices.
    One step = forward + loss + backward + flat all-reduce + AdamW (hidden 128 / 64, 3 passes)."""
    from argparse import Namespace
    world, rank, local_rank, dev, n_dev, backend = init_dist(args.rehearsal)
    from gnn import cgc, ops
    from gnn.data import collate
    from gnn.parallel import FlatGradAllReduce, broadcast_parameters
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss
    modified = args.model == "cgc_modified"
    hid = 128 if modified else 64
    p = Namespace(hidden_irreps=hid, interaction_reduction="sum", global_reduction="mean",
                  message_passes=3, positive="square")
    ds = SyntheticLattices(args.batch * world, args.nodes, args.edges, 1234)
    batch = collate([ds[rank * args.batch + g] for g in range(args.batch)]).to(dev)
    torch.manual_seed(0)
    model = (cgc.CrystGraphConv if modified else cgc.CrystGraphConvVanilla)(p).to(dev)
    from gnn import EnergyEquivGNN
    EnergyEquivGNN.edge_graph(batch)
    iu = torch.triu_indices(6, 6)
    target = batch.stiffness if modified else batch.stiffness[:, iu[0], iu[1]]
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, amsgrad=True, weight_decay=1e-8)
    broadcast_parameters(model)
    allreduce = FlatGradAllReduce(list(model.parameters()))

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], target)
        loss.backward()
        allreduce()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ops.TIMER.enabled = True
    ops.TIMER.records.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ops.TIMER.enabled = False
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ksum = ops.TIMER.summary()
    if rank == 0:
        n_tot, e_tot = args.batch * args.nodes, args.batch * args.edges
        roof = None
        if "cgc_fwd" in ksum or "cgc_fwd_res" in ksum:
            # the layers with the residual in the store (cgc_fwd_res) read h as well: the
            # launch-weighted bytes over the launch-weighted time of both
            parts = [(ksum[k]["count"], cgc_fwd_bytes(n_tot, e_tot, hid, k == "cgc_fwd_res"),
                      ksum[k]["mean_ms"]) for k in ("cgc_fwd", "cgc_fwd_res") if k in ksum]
            cnt = sum(c for c, _, _ in parts)
            byts = round(sum(c * b for c, b, _ in parts) / cnt)
            ms = sum(c * m for c, _, m in parts) / cnt
            ach = byts / (ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                    "traffic_detail": pmc_traffic("cgc_fwd_kernel", args),
                    "kernel": "cgc_fwd (fused gather + factored edge projection + softplus*sigmoid + segmented sum)",
                    "bytes_per_launch": byts, "mean_ms": round(ms, 4), "launches": cnt}
            if roof["traffic_detail"]:
                roof["traffic"] = roof["traffic_detail"]["bytes"]
                roof["traffic_detail"]["ratio_to_algorithmic"] = round(roof["traffic"] / byts, 3)
        out = {"metric": f"lattice-graphs/s (fwd+bwd), {args.model} 3-layer, ~1k nodes/~4k edges",
               "value": round(world * args.batch * args.steps / dt, 2), "unit": "lattice-graphs/s",
               "n_gpus": n_dev, "ranks": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic periodic lattices (SURVEY 8d generator), random-init weights",
               "config": {"workload": f"{args.model} hidden {hid}, {args.batch} graphs/GPU x "
                                      f"{args.nodes} nodes/{args.edges} edges, fwd+loss+bwd+allreduce+AdamW",
                          "global_batch": args.batch * world, "parallelism": f"graph-sharded dp{world}"},
               "backend": backend, "rehearsal": backend == "gloo",
               "loss": round(float(loss.item()), 6), "roofline": roof, "cpu_baseline": None}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_cgc(modified, p, args.nodes, args.edges, min(args.cpu_budget, 10.0))
        if args.kernel_summary:
            print(json.dumps(ksum, indent=1), file=sys.stderr)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="graphs per GPU per step")
    ap.add_argument("--nodes", type=int, default=1024)
    ap.add_argument("--edges", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--lmax", type=int, default=4)
    ap.add_argument("--correlation", type=int, default=3, choices=[1, 2, 3, 4],
                    help="symmetric-contraction correlation (4: the table-driven kernels, lmax <= 3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=25.0)
    ap.add_argument("--cpu-full", action="store_true",
                    help="(default) CPU baseline with BASELINE.md section 2's 3 warm-up + 10 timed steps")
    ap.add_argument("--cpu-quick", action="store_true",
                    help="CPU baseline with 1 warm-up + timed steps within --cpu-budget (at least 1)")
    ap.add_argument("--kernel-summary", action="store_true", help="print per-kernel timings to stderr")
    ap.add_argument("--inline-steps", type=int, default=5,
                    help="in-line steps after the timed region whose tp_fwd launch time gives the "
                         "roofline (0: the overlapped timed region's own figure)")
    ap.add_argument("--model", default="egnn", choices=["egnn", "cgc_modified", "cgc_vanilla"],
                    help="egnn = the headline EnergyEquivGNN; cgc_* = BASELINE config 4 benchmark models")
    ap.add_argument("--optimizer", default="fused", choices=["fused", "foreach"],
                    help="AdamW implementation (same update rule)")
    ap.add_argument("--storage", default="float32", choices=["float32", "bfloat16"],
                    help="storage type of the edge-sized interaction tensors (fp32 arithmetic)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="N > 1 ranks on fewer GPUs (shared devices, gloo): exercises the multi-rank "
                         "path; the line is labelled a rehearsal, not a multi-GPU measurement")
    ap.add_argument("--check-params", action="store_true",
                    help="N > 1: check after the timed steps that every rank holds bitwise-equal "
                         "parameters (reported as params_equal_across_ranks)")
    ap.add_argument("--node-order", default="none", choices=["none", "morton", "auto"],
                    help="collate-time node numbering within each graph: as generated, Morton "
                         "(Z-order of the positions), or auto = Morton for graphs over 2048 nodes")
    ap.add_argument("--config", type=int, default=2, choices=[2, 5],
                    help="2 = BASELINE configs[1] (default); 5 = configs[4]: lmax 3, ~5k-node "
                         "lattices (5000 nodes / 20000 edges), bf16 storage, fp32 accumulate")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; "
              "using WORLD_SIZE", file=sys.stderr)
    if args.config == 5:
        args.lmax, args.nodes, args.edges, args.storage = 3, 5000, 20000, "bfloat16"
    if args.model != "egnn":
        return main_cgc(args)

    world, rank, local_rank, dev, n_dev, backend = init_dist(args.rehearsal)

    from gnn import EnergyEquivGNN, ops
    from gnn.data import collate
    from gnn.synthetic import SyntheticLattices
    from gnn.train import stiffness_loss

    # graphs rank*B .. rank*B+B-1 (graph-sharded, seed 1234 + global graph id)
    ds = SyntheticLattices(args.batch * world, args.nodes, args.edges, 1234)
    mine = [ds[rank * args.batch + g] for g in range(args.batch)]
    if args.node_order == "morton" or (args.node_order == "auto" and args.nodes > 2048):
        from gnn.data import morton_order, reorder_nodes
        mine = [reorder_nodes(d, morton_order(d.positions)) for d in mine]
        args.node_order = "morton"
    else:
        args.node_order = "as generated"
    rmax = torch.tensor([max(float(d.edge_attr.max()) for d in mine)], device=dev)
    if world > 1:
        dist.all_reduce(rmax, op=dist.ReduceOp.MAX)
    params = make_params(args.layers, float(rmax.item()), args.lmax, args.storage, args.correlation)
    torch.manual_seed(0)
    model = EnergyEquivGNN(params).to(dev)
    # AdamW(amsgrad) as the reference configures it (scripts/train_utils.py:39-43); the fused
    # multi-tensor kernel is the same update in one launch per parameter group
    opt = torch.optim.AdamW(model.parameters(), lr=params.lr, betas=(params.beta1, 0.999),
                            eps=params.epsilon, amsgrad=params.amsgrad, weight_decay=params.weight_decay,
                            **({"fused": True} if args.optimizer == "fused" else {"foreach": True}))
    batch = collate(mine).to(dev)
    model.edge_graph(batch)     # CSR built once per batch (collate-time work)
    from gnn.parallel import FlatGradAllReduce, broadcast_parameters
    broadcast_parameters(model)
    plist = [p for p in model.parameters()]
    allreduce = FlatGradAllReduce(plist)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = stiffness_loss(model(batch)["stiffness"], batch.stiffness)
        loss.backward()
        allreduce()                      # one flat fp32 RCCL all-reduce (no-op at N=1)
        torch.nn.utils.clip_grad_norm_(plist, 10.0)
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ops.TIMER.enabled = True
    ops.TIMER.records.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ops.TIMER.enabled = False
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ksum = ops.TIMER.summary()
    same = params_equal_across_ranks(plist) if (world > 1 and args.check_params) else None
    # the roofline kernel's launch time in the in-line step (every kernel on the main stream,
    # EELG_OVERLAP=0's order), after the timed region: the figure a rocprofv3 kernel trace of
    # this command reproduces (profiles/r08a_frac_probe.md); the overlapped timed region's own
    # HIP-event figure is reported beside it
    ksum_inl = inline_kernel_times(step, args.inline_steps) if args.inline_steps > 0 else {}

    if rank == 0:
        n_tot = args.batch * args.nodes
        e_tot = args.batch * args.edges
        key = "tp_fwd[din=800]" if args.lmax == 4 else "tp_fwd[din=512]"
        lay = model.stiffness_head.layers[1].interaction
        info = lay._config()[1]
        roof = None
        if key in ksum:
            byts = tp_fwd_bytes(n_tot, e_tot, info["din"], info["wn"], info["dmid"], info["nsh"],
                                2 if args.storage == "bfloat16" else 4)
            ovl = {"mean_ms": round(ksum[key]["mean_ms"], 4), "launches": ksum[key]["count"],
                   "frac": round(byts / (ksum[key]["mean_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                   "timing": "HIP events on the launch stream over the timed region (side-stream "
                             "overlap on, the step the value is measured on)"}
            src = ksum_inl if key in ksum_inl else ksum
            ms = src[key]["mean_ms"]
            ach = byts / (ms * 1e-3) / 1e9
            # the generated kernel's name (the bf16-storage form carries the _bw suffix)
            kname = f"tp_fwd_tpB_l{args.lmax}" + ("_bw" if args.storage == "bfloat16" else "")
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4),
                    "traffic": None, "traffic_detail": pmc_traffic(kname, args),
                    "kernel": f"{kname} (fused gather+TP+segmented sum)",
                    "bytes_per_launch": byts, "mean_ms": round(ms, 4), "launches": src[key]["count"],
                    "timing": ("HIP events on the launch stream, in-line step (EELG_OVERLAP=0 order, "
                               f"{args.inline_steps} steps after the timed region): agrees with the "
                               "rocprofv3 kernel trace of this command, profiles/r08a_frac_probe.md"
                               if src is ksum_inl else ovl["timing"]),
                    "overlapped": ovl}
            if roof["traffic_detail"]:
                roof["traffic"] = roof["traffic_detail"]["bytes"]      # HBM bytes per launch (PMC)
                # measured HBM bytes over the SURVEY 8d algorithmic bytes (x is gathered once per
                # in-edge, not once per node, so > 1 is expected for a gather)
                roof["traffic_detail"]["ratio_to_algorithmic"] = round(roof["traffic"] / byts, 3)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.nodes, args.edges, args.layers, args.cpu_budget, args.lmax,
                               full=not args.cpu_quick, correlation=args.correlation)
        value = world * args.batch * args.steps / dt
        out = {
            "metric": ("lattice-graphs/s (fwd+bwd), 4-layer EnergyEquivGNN, ~1k nodes/~4k edges, 1/2/4/8 GPU"
                       if args.config == 2 else
                       "lattice-graphs/s (fwd+bwd), 4-layer EnergyEquivGNN lmax 3, ~5k nodes/~20k edges, "
                       "bf16 storage + fp32 accumulate (BASELINE configs[4])"),
            "value": round(value, 2), "unit": "lattice-graphs/s", "n_gpus": n_dev, "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if args.storage == "float32" else "f32 (bf16 storage of w / grad_w / gxe)",
            "data": "synthetic periodic lattices (SURVEY 8d generator), random-init weights",
            "config": {"workload": f"EnergyEquivGNN {args.layers}-layer lmax{args.lmax} "
                                   + (f"correlation {args.correlation} " if args.correlation != 3 else "")
                                   + f"({args.storage} edge storage), "
                                   f"{args.batch} graphs/GPU x {args.nodes} nodes/{args.edges} edges, "
                                   "fwd+loss+bwd+allreduce+clip+AdamW",
                       "global_batch": args.batch * world, "nodes_per_graph": args.nodes,
                       "edges_per_graph": args.edges, "layers": args.layers,
                       "correlation": args.correlation, "node_order": args.node_order,
                       "parallelism": f"graph-sharded dp{world}"},
            "backend": backend, "rehearsal": backend == "gloo",
            "loss": round(float(loss.item()), 6),
            "roofline": roof,
            "cpu_baseline": cpu,
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
        }
        if same is not None:
            out["params_equal_across_ranks"] = same
        if args.kernel_summary:
            print(json.dumps(ksum, indent=1), file=sys.stderr)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
