"""Graph-batch data parallelism: one process per GPU, RCCL over xGMI.

Inductive datasets (PPI, PATTERN) are disjoint unions of graphs, so a rank takes its own graphs
(`shard_graphs`, DistributedSampler-equivalent) and the GAT forward needs no communication.
Training needs exactly one exchange per step: the gradient all-reduce (`allreduce_gradients`,
flattened into large buckets — PPI's 1.87 M parameters are one 7.47 MB bucket, which xGMI moves
in tens of microseconds; tiny per-tensor all-reduces would be latency-bound).
`collate_graphs` replaces PyG's `Batch` collate (`models/GATModel.py:273-287` use PyG
DataLoaders, which are not installable here).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import torch
import torch.distributed as dist


def shard_graphs(num_graphs: int, rank: int, world: int) -> List[int]:
    """Graph ids owned by `rank`: r, r+world, ... (every graph exactly once over the ranks)."""
    return list(range(rank, num_graphs, world))


def collate_graphs(graphs: Sequence[tuple]):
    """[(x_i (n_i, F), edge_index_i (2, e_i), y_i or None)] -> (x, edge_index, y, node_offsets):
    node features concatenated, edge ids shifted by the preceding graphs' node counts."""
    xs, eis, ys, offs = [], [], [], [0]
    for g in graphs:
        x, ei = g[0], g[1]
        xs.append(x)
        eis.append(ei + offs[-1])
        if len(g) > 2 and g[2] is not None:
            ys.append(g[2])
        offs.append(offs[-1] + x.shape[0])
    x = torch.cat(xs, 0)
    ei = torch.cat(eis, 1)
    y = torch.cat(ys, 0) if ys else None
    return x, ei, y, torch.tensor(offs, dtype=torch.int64)


def allreduce_gradients(params: Iterable[torch.nn.Parameter], world: int | None = None,
                        bucket_bytes: int = 64 << 20, group=None) -> None:
    """Average .grad across ranks: grads flattened into <= bucket_bytes buckets, one all-reduce
    (SUM) per bucket, scaled by 1/world, copied back. Parameters without grads are skipped (the
    same set on every rank, as in DDP)."""
    if world is None:
        world = dist.get_world_size(group)
    if world == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    bucket, size = [], 0
    for g in grads + [None]:
        if g is not None and (size + g.numel() * g.element_size() <= bucket_bytes or not bucket):
            bucket.append(g)
            size += g.numel() * g.element_size()
            continue
        if bucket:
            flat = torch.cat([b.reshape(-1) for b in bucket])
            if flat.is_cuda and dist.get_backend(group) != "nccl":   # gloo: host staging
                host = flat.cpu()
                dist.all_reduce(host, group=group)
                flat.copy_(host)
            else:
                dist.all_reduce(flat, group=group)
            flat.mul_(1.0 / world)
            off = 0
            for b in bucket:
                n = b.numel()
                b.copy_(flat[off:off + n].view_as(b))
                off += n
        bucket, size = ([g], g.numel() * g.element_size()) if g is not None else ([], 0)
