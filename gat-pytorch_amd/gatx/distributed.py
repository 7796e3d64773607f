"""Graph-batch data parallelism: one process per GPU, RCCL over xGMI.

Inductive datasets (PPI, PATTERN) are disjoint unions of graphs, so a rank takes its own graphs
(`shard_graphs`, DistributedSampler-equivalent) and the GAT forward needs no communication.
Training needs exactly one exchange per step: the gradient all-reduce. `GradientAllReducer`
overlaps it with the backward the way DDP does: gradients are grouped into buckets in reverse
registration order (the order backward produces them), and each bucket's all-reduce is launched
asynchronously from a post-accumulate-grad hook once its gradients are ready (buckets go out in
index order on every rank, whatever order the hooks fire in), while
autograd keeps computing earlier layers' gradients. PPI's 1.87 M parameters (7.47 MB) make a few
buckets; PATTERN's 20 k parameters (81 KB) one latency-bound bucket.

Loss semantics: the reference's losses are means over nodes (BCE, `models/ppi_gat.py:11`,
`models/pattern_gat.py:15`) or edges (`calc_attention_norm`, `models/GATModel.py:224`). With
uneven shards a plain 1/world average of per-rank means is not the union batch's mean; scale each
rank's loss by `count_weight(n_local)` = n_local / n_global (an all-reduce of one scalar) and SUM
the gradients (`average=False`): the result equals one process training on the union batch.

`collate_graphs` replaces PyG's `Batch` collate (`models/GATModel.py:273-287` use PyG
DataLoaders, which are not installable here); `DeviceGraphLoader` is the sampler-driven device
loop built on it.
"""
from __future__ import annotations

import contextlib
from typing import Iterable, List, Sequence

import torch
import torch.distributed as dist


def shard_graphs(num_graphs: int, rank: int, world: int) -> List[int]:
    """Graph ids owned by `rank`: r, r+world, ... (every graph exactly once over the ranks)."""
    return list(range(rank, num_graphs, world))


def collate_graphs(graphs: Sequence[tuple]):
    """[(x_i (n_i, F), edge_index_i (2, e_i), y_i or None)] -> (x, edge_index, y, node_offsets):
    node features concatenated, edge ids shifted by the preceding graphs' node counts. Works on
    whichever device the graphs live on (a device batch needs no host round trip)."""
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


class DeviceGraphLoader:
    """Per-rank batches of whole graphs, resident on the device: each epoch shuffles the graph ids
    with a seed shared by every rank (DistributedSampler semantics: same permutation everywhere,
    the id list padded by wrapping around to a multiple of `world` — or truncated to one with
    drop_last — then rank r takes every world-th id), and collates `batch_size` graphs at a time
    on the device. Every rank therefore yields the same number of batches, so every rank issues
    the same collectives per epoch. `graphs` is a list of (x, edge_index, y) already on the
    device."""

    def __init__(self, graphs, batch_size: int, rank: int = 0, world: int = 1,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if not graphs:
            raise ValueError("DeviceGraphLoader: no graphs")
        if not 0 <= rank < world:
            raise ValueError(f"DeviceGraphLoader: rank {rank} outside world {world}")
        self.graphs, self.batch_size = graphs, batch_size
        self.rank, self.world, self.shuffle, self.seed = rank, world, shuffle, seed
        self.drop_last = drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _ids(self):
        n = len(self.graphs)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(n, generator=g).tolist()
        else:
            order = list(range(n))
        if self.drop_last:
            order = order[:n - n % self.world] if n >= self.world else order[:0]
        else:   # wrap around (repeating as often as needed when n < world)
            total = -(-n // self.world) * self.world
            order = (order * (-(-total // n)))[:total]
        return [order[i] for i in shard_graphs(len(order), self.rank, self.world)]

    def __iter__(self):
        ids = self._ids()
        bs = self.batch_size
        stop = len(ids) - (len(ids) % bs if self.drop_last else 0)
        for i in range(0, stop, bs):
            yield collate_graphs([self.graphs[j] for j in ids[i:i + bs]])

    def __len__(self):
        n = len(self._ids())
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)


def count_weights(counts, group=None, device=None, always_reduce: bool = False):
    """[n_local / sum over ranks of n_local] for each count in `counts`, with ONE all-reduce of
    the vector: the factors that turn this rank's mean loss terms into their shares of the union
    batch's means (SUM the gradients afterwards). Weight each term by its own count — nodes (or
    labelled rows) for BCE / cross-entropy, edges E' for calc_attention_norm (a per-edge mean,
    `models/GATModel.py:224`) — and compute the weights once, outside a captured or timed step
    (this blocks on the result). `always_reduce` runs the collective even at world size 1 (tests
    exercising the RCCL path on a one-GPU box)."""
    counts = [float(c) for c in counts]
    if not dist.is_initialized() or (dist.get_world_size(group) == 1 and not always_reduce):
        return [1.0] * len(counts)
    if device is None:
        device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor(counts, dtype=torch.float64, device=device)
    dist.all_reduce(t, group=group)
    tot = t.cpu().tolist()
    return [c / s if s else 0.0 for c, s in zip(counts, tot)]


def count_weight(n_local: int | float, group=None, device=None,
                 always_reduce: bool = False) -> float:
    """count_weights for a single loss term (a node-mean loss such as PatternGAT's BCE)."""
    return count_weights([n_local], group, device, always_reduce)[0]


def _all_reduce_flat(flat: torch.Tensor, group, async_op: bool):
    if flat.is_cuda and dist.get_backend(group) != "nccl":   # gloo: host staging
        host = flat.cpu()
        dist.all_reduce(host, group=group)
        flat.copy_(host)
        return None
    return dist.all_reduce(flat, group=group, async_op=async_op)


def allreduce_gradients(params: Iterable[torch.nn.Parameter], world: int | None = None,
                        bucket_bytes: int = 64 << 20, group=None, average: bool = True) -> None:
    """Post-hoc all-reduce of .grad across ranks: grads flattened into <= bucket_bytes buckets,
    one all-reduce (SUM) per bucket, scaled by 1/world when `average`, copied back. Parameters
    without grads are skipped (the same set on every rank, as in DDP). GradientAllReducer is the
    overlapped form used by training loops."""
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
            _all_reduce_flat(flat, group, async_op=False)
            if average:
                flat.mul_(1.0 / world)
            off = 0
            for b in bucket:
                n = b.numel()
                b.copy_(flat[off:off + n].view_as(b))
                off += n
        bucket, size = ([g], g.numel() * g.element_size()) if g is not None else ([], 0)


class GradientAllReducer:
    """DDP-style gradient all-reduce overlapped with the backward.

        reducer = GradientAllReducer(model.parameters())
        loss.backward()          # buckets are all-reduced (async) as their gradients land
        reducer.finish()         # wait, write the reduced gradients back into .grad
        opt.step()

    Buckets hold consecutive parameters in reverse registration order (backward produces the
    last layer's gradients first), at most `bucket_bytes` each. A bucket's flat buffer is filled
    from the post-accumulate-grad hooks of its parameters; once the last one has arrived the
    bucket's all-reduce (SUM; then x 1/world when `average`) is issued with async_op, so RCCL
    moves it over xGMI while autograd continues.

    Collective order: RCCL matches collectives by issue order, so every rank must issue the
    buckets' all-reduces in the same order. Buckets are launched strictly in index order, as DDP
    does: a bucket that fills before its predecessors waits in the queue and goes out right after
    them. The order in which autograd fires the hooks may therefore differ between ranks without
    mismatching collectives.

    Parameters whose hook did not fire in the synced backward are filled in finish() from their
    .grad (what no_sync() micro-steps accumulated on this rank) or with zeros when they have none
    (every rank issues the same collectives, as DDP with find_unused_parameters); they leave
    finish() with the reduced .grad (zeros if no rank produced one)."""

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_bytes: int = 4 << 20,
                 group=None, average: bool = True, always_reduce: bool = False):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.average = average
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # always_reduce: hooks and collectives even at world size 1 (tests of the RCCL path on
        # a one-GPU box; a one-rank all-reduce is the identity)
        self.active = self.world > 1 or (always_reduce and dist.is_initialized())
        self._sync = True
        self.buckets: List[dict] = []
        cur, size = [], 0
        for p in reversed(self.params):
            nb = p.numel() * p.element_size()
            if cur and size + nb > bucket_bytes:
                self.buckets.append(self._bucket(cur))
                cur, size = [], 0
            cur.append(p)
            size += nb
        if cur:
            self.buckets.append(self._bucket(cur))
        self._slot = {}
        for bi, b in enumerate(self.buckets):
            for pi, p in enumerate(b["params"]):
                self._slot[id(p)] = (bi, pi)
        self._hooks = []
        if self.active:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset()

    def _bucket(self, params):
        offs, o = [], 0
        for p in params:
            offs.append(o)
            o += p.numel()
        return {"params": params, "offsets": offs, "numel": o, "flat": None}

    def _reset(self):
        self._next = 0   # the next bucket to launch (buckets go out in index order)
        for b in self.buckets:
            b["ready"] = 0
            b["work"] = None
            b["launched"] = False
            b["seen"] = [False] * len(b["params"])

    def _flat(self, b, like):
        if b["flat"] is None or b["flat"].device != like.device:
            b["flat"] = torch.zeros(b["numel"], dtype=like.dtype, device=like.device)
        return b["flat"]

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation (DDP's no_sync): backward passes inside the context only
        accumulate into .grad; the first backward after it reduces the accumulated gradients.
        Call finish() once, after that backward."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _on_grad(self, p):
        if not self._sync:
            return
        bi, pi = self._slot[id(p)]
        b = self.buckets[bi]
        if b["launched"]:
            # a second backward before finish(): the bucket's all-reduce is already in flight
            # (or done) on the old values; refilling its buffer would race with it and the new
            # contribution would never be reduced
            raise RuntimeError("GradientAllReducer: backward ran twice before finish(); use "
                               "no_sync() for the accumulation steps")
        flat = self._flat(b, p.grad)
        o = b["offsets"][pi]
        flat[o:o + p.numel()].copy_(p.grad.reshape(-1))
        if not b["seen"][pi]:
            b["seen"][pi] = True
            b["ready"] += 1
        self._launch_ready()

    def _launch(self, b):
        b["launched"] = True
        b["work"] = _all_reduce_flat(b["flat"], self.group, async_op=True)
        self._next += 1

    def _launch_ready(self):
        """Issue the all-reduces of the complete buckets at the head of the queue, in index
        order (never a later bucket ahead of an earlier one: the collective order is the same on
        every rank whatever order the hooks fired in)."""
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if b["ready"] != len(b["params"]):
                return
            self._launch(b)

    def finish(self):
        """Wait for every bucket's all-reduce and write the results into .grad."""
        if not self.active:
            return
        dev = next((p.grad.device for p in self.params if p.grad is not None), None)
        for b in self.buckets:   # the rest of the queue, still in index order
            if b["launched"]:
                continue
            flat = self._flat(b, torch.empty(0, device=dev) if dev is not None
                              else b["params"][0])
            for pi, p in enumerate(b["params"]):
                if not b["seen"][pi]:
                    # no hook in the synced backward: this rank's gradient is whatever .grad
                    # holds (no_sync() micro-steps), or nothing
                    o = b["offsets"][pi]
                    if p.grad is not None:
                        flat[o:o + p.numel()].copy_(p.grad.reshape(-1))
                    else:
                        flat[o:o + p.numel()].zero_()
            self._launch(b)
        for b in self.buckets:
            if b["work"] is not None:
                b["work"].wait()
            flat = b["flat"]
            if self.average:
                flat.mul_(1.0 / self.world)
            for pi, p in enumerate(b["params"]):
                o = b["offsets"][pi]
                v = flat[o:o + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = v.clone()
                else:
                    p.grad.copy_(v)
        self._reset()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
