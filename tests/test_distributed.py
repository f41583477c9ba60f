"""Graph-sharded data parallelism on CPU with gloo, world sizes 2 and 8 (SURVEY.md 4.5, 8e;
8 = BASELINE config 3's rank count, ``scripts/train_main.py:89-100``).

Checks that sharding whole graphs across ranks + one flat gradient all-reduce
(``gnn.parallel.FlatGradAllReduce``) reproduces the single-process full-batch
gradient, and that ``broadcast_parameters`` syncs replicas.  The model here is
the CPU oracle (the parallel logic is model-agnostic; the HIP model runs the same
code path with backend 'nccl' = RCCL in ``bench.py``)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import batch_to
from test_oracle import small_params


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graphs(n=4):
    from gnn.synthetic import SyntheticLattices
    return SyntheticLattices(n, 24, 96, 77)


def _model(seed):
    import oracle.model as omodel
    torch.manual_seed(seed)
    return omodel.EnergyEquivGNN(small_params(max_edge_radius=_graphs().max_edge_radius)).double()


def _worker(rank, world, port, out, per_rank=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from gnn.data import collate
    from gnn.parallel import FlatGradAllReduce, broadcast_parameters, shard_indices
    from oracle.train import stiffness_loss
    m = _model(seed=rank + 100)          # deliberately different init per rank
    broadcast_parameters(m)              # -> rank 0's weights everywhere
    ds = _graphs(world * per_rank)
    idx = shard_indices(len(ds), rank, world, per_rank=per_rank)
    b = batch_to(collate([ds[i] for i in idx]), "cpu", torch.float64)
    loss = stiffness_loss(m(b)["stiffness"], b.stiffness)
    loss.backward()
    FlatGradAllReduce(m.parameters())()
    if rank == 0:
        torch.save({k: p.grad.clone() for k, p in m.named_parameters()}, out)
        torch.save({k: p.detach().clone() for k, p in m.named_parameters()}, out + ".w")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank", [(2, 2), (8, 1)])
def test_sharded_allreduce_matches_full_batch_gradient(world, per_rank):
    """``world`` gloo ranks, each with ``per_rank`` whole graphs and its own init (replaced by
    rank 0's through ``broadcast_parameters``): after one flat all-reduce rank 0's averaged
    gradient equals the single-process gradient of the whole ``world * per_rank``-graph batch."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "grads.pt")
        mp.spawn(_worker, args=(world, _free_port(), out, per_rank), nprocs=world, join=True)
        grads = torch.load(out, weights_only=True)
        weights = torch.load(out + ".w", weights_only=True)
    from gnn.data import collate
    from oracle.train import stiffness_loss
    m = _model(seed=100)                 # rank 0's init
    for k, p in m.named_parameters():
        assert torch.equal(p.detach(), weights[k]), k
    ds = _graphs(world * per_rank)
    b = batch_to(collate([ds[i] for i in range(world * per_rank)]), "cpu", torch.float64)
    loss = stiffness_loss(m(b)["stiffness"], b.stiffness)
    loss.backward()
    for k, p in m.named_parameters():
        err = float((p.grad - grads[k]).abs().max() / p.grad.abs().max().clamp_min(1e-300))
        assert err < 1e-6, (k, err)      # reduction-order noise only; a wrong all-reduce is O(1)


def test_shard_indices_partition_the_global_batch():
    from gnn.parallel import shard_indices
    world, per = 4, 3
    got = sorted(i for r in range(world) for i in shard_indices(100, r, world, per, step=2))
    assert got == list(range(24, 36))
