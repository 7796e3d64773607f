"""Multi-process checks of the graph-batch data-parallel path on CPU (gloo, world_size 2): the
sharding covers every graph once, collate matches a PyG-style batch, and the bucketed gradient
all-reduce gives every rank the average of the per-rank gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gatx.distributed import allreduce_gradients, collate_graphs, shard_graphs


def test_shard_graphs_partition():
    for n, w in [(20, 2), (20, 8), (7, 4), (3, 8)]:
        got = sorted(g for r in range(w) for g in shard_graphs(n, r, w))
        assert got == list(range(n))


def test_collate_offsets():
    g1 = (torch.ones(3, 2), torch.tensor([[0, 1], [1, 2]]), torch.zeros(3))
    g2 = (torch.zeros(2, 2), torch.tensor([[1], [0]]), torch.ones(2))
    x, ei, y, offs = collate_graphs([g1, g2])
    assert x.shape == (5, 2) and y.shape == (5,)
    assert ei.tolist() == [[0, 1, 4], [1, 2, 3]]
    assert offs.tolist() == [0, 3, 5]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bucket, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 3))
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(11, 5, generator=g)
    model(x).square().sum().backward()
    allreduce_gradients(model.parameters(), bucket_bytes=bucket)
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket", [64 << 20, 64])
def test_allreduce_gradients_gloo_world2(bucket):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), bucket, out), nprocs=world, join=True)
    # single-process reference: average of the per-rank gradients
    ref = []
    for r in range(world):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 3))
        x = torch.randn(11, 5, generator=torch.Generator().manual_seed(100 + r))
        model(x).square().sum().backward()
        ref.append(torch.cat([p.grad.reshape(-1) for p in model.parameters()]))
    avg = sum(ref) / world
    for r in range(world):
        assert torch.allclose(out[r], avg, atol=1e-6)
