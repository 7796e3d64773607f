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
    """DistributedSampler semantics: 7 graphs over 3 ranks pad to 9 ids by wrapping around, so
    every rank yields the same number of batches (same collectives per epoch) and every graph is
    seen at least once."""
    from gatx.distributed import DeviceGraphLoader
    graphs = [(torch.full((2, 1), float(i)), torch.tensor([[0], [1]]), None) for i in range(7)]
    seen, lens, nbatches = [], [], []
    for r in range(3):
        ld = DeviceGraphLoader(graphs, batch_size=2, rank=r, world=3, seed=4)
        ld.set_epoch(1)
        lens.append(len(ld))
        k = 0
        for x, ei, _, offs in ld:
            seen += x[::2, 0].int().tolist()
            assert ei.shape[1] == len(offs) - 1
            k += 1
        nbatches.append(k)
    assert len(set(lens)) == 1 and lens == nbatches == [2, 2, 2]
    assert sorted(set(seen)) == list(range(7)) and len(seen) == 9


@pytest.mark.parametrize("n,world,bs", [(7, 3, 2), (2, 4, 1), (8, 3, 3), (5, 5, 2)])
def test_device_graph_loader_equal_lengths(n, world, bs):
    from gatx.distributed import DeviceGraphLoader
    graphs = [(torch.full((1, 1), float(i)), torch.zeros((2, 0), dtype=torch.int64), None)
              for i in range(n)]
    for drop_last in (False, True):
        lens = [len(DeviceGraphLoader(graphs, bs, r, world, drop_last=drop_last))
                for r in range(world)]
        assert len(set(lens)) == 1, (drop_last, lens)
        got = [len(list(DeviceGraphLoader(graphs, bs, r, world, drop_last=drop_last)))
               for r in range(world)]
        assert got == lens
        if drop_last:
            ids = sorted(int(x[0, 0]) for r in range(world)
                         for x, _, _, _ in DeviceGraphLoader(graphs, 1, r, world,
                                                             drop_last=True))
            assert len(ids) == len(set(ids)) == n - n % world


def _accum_worker(rank, world, port, out):
    """Gradient accumulation: two micro-batches under no_sync + a third outside it, one
    finish(); and a second backward before finish() must raise (not silently mix gradients)."""
    from gatx.distributed import GradientAllReducer, count_weights
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 1))
    reducer = GradientAllReducer(model.parameters(), bucket_bytes=64, average=False)
    x, y = _union_data()
    # rank r's micro-batches: rows r, r+world, ... cut into three
    rows = list(range(rank, 13, world))
    parts = [rows[0::3], rows[1::3], rows[2::3]]
    w = count_weights([len(rows)])[0]
    model.zero_grad(set_to_none=True)
    for i, part in enumerate(parts):
        loss = torch.nn.functional.binary_cross_entropy_with_logits(
            model(x[part]).squeeze(-1), y[part], reduction="sum") / len(rows)
        if i < 2:
            with reducer.no_sync():
                (loss * w).backward()
        else:
            (loss * w).backward()
    reducer.finish()
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    model(x[rows]).sum().backward()
    try:
        model(x[rows]).sum().backward()
    except RuntimeError as e:
        out[f"err{rank}"] = "twice before finish" in str(e)
    else:
        out[f"err{rank}"] = False
    reducer.remove()
    dist.destroy_process_group()


def test_gradient_accumulation_no_sync_world3():
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_accum_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 1))
    x, y = _union_data()
    torch.nn.functional.binary_cross_entropy_with_logits(model(x).squeeze(-1), y).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    for r in range(world):
        assert torch.allclose(out[r], ref, atol=1e-6), (r, (out[r] - ref).abs().max())
        assert out[f"err{r}"], r


def _two_term_worker(rank, world, port, out):
    """Two mean terms over different counts (a node-mean BCE plus an edge-mean term, as
    PPI_GAT's BCE + attention_penalty * calc_attention_norm): each weighted by its own count."""
    from gatx.distributed import GradientAllReducer, count_weights
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 1))
    reducer = GradientAllReducer(model.parameters(), average=False)
    x, y = _union_data()
    rows = [list(range(0, 3)), list(range(3, 8)), list(range(8, 13))][rank]
    edges = [list(range(0, 2)), list(range(2, 9)), list(range(9, 13))][rank]   # uneven, != rows
    w_n, w_e = count_weights([len(rows), len(edges)])
    bce = torch.nn.functional.binary_cross_entropy_with_logits(model(x[rows]).squeeze(-1), y[rows])
    pen = model(x[edges]).abs().mean()
    (bce * w_n + 0.3 * pen * w_e).backward()
    reducer.finish()
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    reducer.remove()
    dist.destroy_process_group()


def test_per_term_count_weights_world3():
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_two_term_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.ELU(), torch.nn.Linear(7, 1))
    x, y = _union_data()
    (torch.nn.functional.binary_cross_entropy_with_logits(model(x).squeeze(-1), y)
     + 0.3 * model(x).abs().mean()).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    for r in range(world):
        assert torch.allclose(out[r], ref, atol=1e-6), (r, (out[r] - ref).abs().max())


class _TwoBranch(torch.nn.Module):
    """out = branch_a(x) + branch_b(x). `b_first` evaluates branch_b first: autograd then runs
    branch_a's backward first (reverse creation order), so the parameters' post-accumulate-grad
    hooks fire in a different order with the same values (float addition commutes)."""

    def __init__(self):
        super().__init__()
        self.a1, self.a2 = torch.nn.Linear(5, 6), torch.nn.Linear(6, 1)
        self.b1, self.b2 = torch.nn.Linear(5, 4), torch.nn.Linear(4, 1)

    def branch_a(self, x):
        return self.a2(torch.nn.functional.elu(self.a1(x)))

    def branch_b(self, x):
        return self.b2(torch.nn.functional.elu(self.b1(x)))

    def forward(self, x, b_first=False, use=("a", "b")):
        if use == ("a",):
            return self.branch_a(x)
        if use == ("b",):
            return self.branch_b(x)
        if b_first:
            yb = self.branch_b(x)
            return self.branch_a(x) + yb
        ya = self.branch_a(x)
        return ya + self.branch_b(x)


def _order_worker(rank, world, port, out):
    """Rank 1 fires its hooks in another order than ranks 0 and 2 (one bucket per parameter):
    the buckets must still go out in index order everywhere, giving the union-batch gradient."""
    from gatx.distributed import GradientAllReducer, count_weight
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = _TwoBranch()
    fired = []
    for name, p in model.named_parameters():
        p.register_post_accumulate_grad_hook(lambda p, n=name: fired.append(n))
    reducer = GradientAllReducer(model.parameters(), bucket_bytes=64, average=False)
    x, y = _union_data()
    rows = [list(range(0, 3)), list(range(3, 8)), list(range(8, 13))][rank]
    for _ in range(2):
        fired.clear()
        model.zero_grad(set_to_none=True)
        w = count_weight(len(rows))
        loss = torch.nn.functional.binary_cross_entropy_with_logits(
            model(x[rows], b_first=rank == 1).squeeze(-1), y[rows])
        (loss * w).backward()
        reducer.finish()
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    out[f"fired{rank}"] = list(fired)
    out[f"nbuckets{rank}"] = len(reducer.buckets)
    reducer.remove()
    dist.destroy_process_group()


def test_bucket_order_independent_of_hook_order_world3():
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_order_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    # the permutation really happened: rank 1's hooks fired in another order
    assert out["fired0"] == out["fired2"] and out["fired0"] != out["fired1"]
    assert out["nbuckets0"] >= 4
    torch.manual_seed(0)
    model = _TwoBranch()
    x, y = _union_data()
    torch.nn.functional.binary_cross_entropy_with_logits(model(x).squeeze(-1), y).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    for r in range(world):
        assert torch.allclose(out[r], ref, atol=1e-6), (r, (out[r] - ref).abs().max())


def _nosync_only_worker(rank, world, port, out):
    """branch_b gets its gradient only in the no_sync micro-step; the synced backward touches
    branch_a alone. finish() must reduce branch_b's accumulated .grad, not zeros."""
    from gatx.distributed import GradientAllReducer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = _TwoBranch()
    reducer = GradientAllReducer(model.parameters(), bucket_bytes=64, average=False)
    x, _ = _union_data()
    rows = list(range(rank, 13, world))
    model.zero_grad(set_to_none=True)
    with reducer.no_sync():
        model(x[rows], use=("b",)).sum().backward()
    model(x[rows], use=("a",)).sum().backward()
    reducer.finish()
    out[rank] = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).clone()
    reducer.remove()
    dist.destroy_process_group()


def test_no_sync_only_gradient_is_reduced_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_nosync_only_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    torch.manual_seed(0)
    model = _TwoBranch()
    x, _ = _union_data()
    model(x, use=("b",)).sum().backward()
    model(x, use=("a",)).sum().backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    for r in range(world):
        assert torch.allclose(out[r], ref, atol=1e-5), (r, (out[r] - ref).abs().max())


# ---------------------------------------------------------------------------------------------
# BASELINE config 4 at 8 ranks: PatternGAT's step (`models/pattern_gat.py:
# 18-25`, batch sharded over the graph axis, `run_config.py:46`) on the reference dataflow
# restated in torch (oracle/torch_dataflow.py, CPU; the HIP layer has no CPU path), through the
# production sharding (shard_graphs / collate_graphs), count_weights and the overlapped
# GradientAllReducer over gloo: every rank's reduced gradient equals one process's gradient on
# the union batch.

def _pattern_params():
    from gatx.config import data_config
    cfg = data_config["PATTERN"]
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    torch.manual_seed(0)
    params = torch.nn.ParameterList()
    for i in range(cfg["num_layers"]):
        fin, F, NH = heads[i] * widths[i], widths[i + 1], heads[i + 1]
        W = torch.empty(NH * F, fin)
        a = torch.empty(NH, NH * 2 * F)
        s = torch.empty(NH * F, fin)
        for t in (W, a, s):
            torch.nn.init.xavier_uniform_(t)
        params.extend([torch.nn.Parameter(W), torch.nn.Parameter(a), torch.nn.Parameter(s)])
    return cfg, params


def _pattern_graphs(num_graphs):
    from gatx import data as gd
    b = gd.dataset_batch("PATTERN", num_graphs, graph_seed=271, feature_seed=16)
    y = (gd.uniform01(28, b.num_nodes) < 0.1765).astype("float32")
    out = []
    for g in range(num_graphs):
        n0, n1 = int(b.node_offsets[g]), int(b.node_offsets[g + 1])
        m = (b.edge_index[1] >= n0) & (b.edge_index[1] < n1)
        out.append((torch.from_numpy(b.x[n0:n1]), torch.from_numpy(b.edge_index[:, m] - n0),
                    torch.from_numpy(y[n0:n1])))
    return out


def _pattern_loss(cfg, params, x, ei, y, w_nodes=1.0, w_edges=1.0):
    from oracle import torch_dataflow as td
    L = cfg["num_layers"]
    layers = [(params[3 * i], params[3 * i + 1]) for i in range(L)]
    skips = [params[3 * i + 2] for i in range(L)]
    out, ei2, alphas = td.model_forward(x, ei, layers, skips, cfg["num_heads_per_layer"],
                                        cfg["head_output_features_per_layer"][1:],
                                        cfg["heads_concat_per_layer"],
                                        cfg["add_skip_connection"])
    bce = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([1 / 0.1765]))(out.squeeze(-1), y)
    # + the attention-norm term (PPI_GAT's attention_penalty form, a per-edge mean), weighted by
    # the rank's share of the union batch's E'
    return bce * w_nodes + 0.5 * td.attention_norm(ei2, alphas) * w_edges, ei2.size(1)


def _pattern_world_worker(rank, world, port, num_graphs, out):
    from gatx.distributed import GradientAllReducer, collate_graphs, count_weights, shard_graphs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, params = _pattern_params()
    reducer = GradientAllReducer(params, bucket_bytes=16 << 10, average=False)
    graphs = _pattern_graphs(num_graphs)
    mine = shard_graphs(num_graphs, rank, world)
    x, ei, y, _ = collate_graphs([graphs[i] for i in mine])
    from oracle import torch_dataflow as td
    e_local = td.self_loop_rewrite(ei).size(1)
    w_n, w_e = count_weights([x.size(0), e_local])
    loss, _ = _pattern_loss(cfg, params, x, ei, y, w_n, w_e)
    loss.backward()
    reducer.finish()
    out[rank] = (len(mine), torch.cat([p.grad.reshape(-1) for p in params]).clone())
    reducer.remove()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("num_graphs", [32, 37])
def test_pattern_sharded_world8_equals_union_batch(num_graphs):
    """32 graphs = 4 per rank (the notebook's PATTERN batch, ipynb:690, over 8 GPUs); 37 graphs
    = uneven 5/5/5/5/5/4/4/4 shards."""
    world = 8
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_pattern_world_worker, args=(world, _free_port(), num_graphs, out), nprocs=world,
             join=True)
    from gatx.distributed import collate_graphs
    cfg, params = _pattern_params()
    x, ei, y, _ = collate_graphs(_pattern_graphs(num_graphs))
    loss, _ = _pattern_loss(cfg, params, x, ei, y)
    loss.backward()
    ref = torch.cat([p.grad.reshape(-1) for p in params])
    sizes = sorted(out[r][0] for r in range(world))
    assert sum(sizes) == num_graphs and sizes[-1] - sizes[0] <= 1
    for r in range(world):
        got = out[r][1]
        assert torch.allclose(got, ref, rtol=1e-4, atol=1e-6), (r, (got - ref).abs().max())
