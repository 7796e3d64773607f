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


def _union_worker(rank, world, port, bucket, out):
    """Uneven shards, per-rank mean loss weighted by count_weight, gradients SUMmed by the
    overlapped GradientAllReducer: must equal one process on the union batch."""
    from gatx.distributed import GradientAllReducer, count_weight
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 3),
                                torch.nn.ELU(), torch.nn.Linear(3, 1))
    reducer = GradientAllReducer(model.parameters(), bucket_bytes=bucket, average=False)
    x, y = _union_data()
    rows = [list(range(0, 4)), list(range(4, 13))][rank]     # 4 vs 9 nodes
    for _ in range(2):   # two steps: the hooks and buckets are reusable
        model.zero_grad(set_to_none=True)
        w = count_weight(len(rows))
        loss = torch.nn.functional.binary_cross_entropy_with_logits(model(x[rows]).squeeze(-1),
                                                                    y[rows])
        (loss * w).backward()
        reducer.finish()
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    reducer.remove()
    dist.barrier()
    dist.destroy_process_group()


def _union_data():
    g = torch.Generator().manual_seed(5)
    return torch.randn(13, 5, generator=g), (torch.rand(13, generator=g) > 0.5).float()


@pytest.mark.parametrize("bucket", [4 << 20, 64])
def test_overlapped_allreduce_equals_union_batch(bucket):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_union_worker, args=(world, _free_port(), bucket, out), nprocs=world, join=True)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 3),
                                torch.nn.ELU(), torch.nn.Linear(3, 1))
    x, y = _union_data()
    torch.nn.functional.binary_cross_entropy_with_logits(model(x).squeeze(-1), y).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    for r in range(world):
        assert torch.allclose(out[r], ref, atol=1e-6), (r, (out[r] - ref).abs().max())


def test_device_graph_loader_partitions_epoch():
    from gatx.distributed import DeviceGraphLoader
    graphs = [(torch.full((2, 1), float(i)), torch.tensor([[0], [1]]), None) for i in range(7)]
    seen = []
    for r in range(3):
        ld = DeviceGraphLoader(graphs, batch_size=2, rank=r, world=3, seed=4)
        ld.set_epoch(1)
        for x, ei, _, offs in ld:
            seen += x[::2, 0].int().tolist()
            assert ei.shape[1] == len(offs) - 1
    assert sorted(seen) == list(range(7))
