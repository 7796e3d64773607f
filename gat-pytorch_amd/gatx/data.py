"""Deterministic synthetic inputs for the GAT hot path.

Everything here is a pure function of integer seeds built on splitmix64, vectorised in numpy, so
the same graph / feature / weight bytes can be regenerated bit-identically in this container (where
the golden fixtures are made) and on the GPU box (where only the expected outputs travel).

Shapes follow SURVEY.md §8(d):
  * uniform per-graph batches (a PyG-style disjoint union: graph g's node ids are offset by the
    node count of graphs < g; edges never cross graphs), used for Cora / PPI / PATTERN shapes;
  * Graph500 R-MAT for the single-graph HBM-roofline case.

The reference gets its graphs from torch_geometric datasets (`models/ppi_gat.py:61-64`,
`models/pattern_gat.py:136-139`, `models/planetoid_gat.py:203-206`) which need a download; no
dataset is available offline, so benchmark inputs are synthetic with the datasets' average sizes.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_MASK64 = (1 << 64) - 1


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """The n uint64 outputs [start, start+n) of splitmix64 seeded with `seed`."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed & _MASK64) + i * _GAMMA
        return _mix(z)


def uniform01(seed: int, n: int, start: int = 0) -> np.ndarray:
    """24-bit uniform floats in [0, 1) (exact in fp32)."""
    return (splitmix64(seed, n, start) >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)


def randint(seed: int, n: int, high, start: int = 0) -> np.ndarray:
    """Uniform integers in [0, high) by multiply-high of the top 32 bits (high may be an array)."""
    hi = splitmix64(seed, n, start) >> np.uint64(32)
    return ((hi * np.asarray(high, dtype=np.uint64)) >> np.uint64(32)).astype(np.int64)


def normal(seed: int, n: int) -> np.ndarray:
    """Standard normal fp32 by Box-Muller on two independent 53-bit uniform streams."""
    u1 = ((splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) + 1.0) * 2.0 ** -53
    u2 = (splitmix64(seed ^ 0x5DEECE66D, n) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def xavier_uniform(seed: int, fan_out: int, fan_in: int) -> np.ndarray:
    """Same distribution as `nn.init.xavier_uniform_` on an (fan_out, fan_in) weight
    (`models/gat_layer.py:142-145`), but drawn from splitmix64 so it is reproducible anywhere."""
    bound = np.sqrt(6.0 / (fan_in + fan_out))
    u = uniform01(seed, fan_out * fan_in).reshape(fan_out, fan_in).astype(np.float64)
    return ((2.0 * u - 1.0) * bound).astype(np.float32)


@dataclass
class GraphBatch:
    """A disjoint union of graphs, PyG `Batch` style: x (N, F_in) fp32, edge_index (2, E) int64."""
    x: np.ndarray
    edge_index: np.ndarray
    num_graphs: int
    node_offsets: np.ndarray  # (G+1,) node id ranges per graph

    @property
    def num_nodes(self) -> int:
        return int(self.x.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])


def uniform_graph_batch(num_graphs: int, nodes_per_graph: int, edges_per_graph: int,
                        in_features: int, graph_seed: int = 42, feature_seed: int = 1,
                        features: str = "normal", bernoulli_p: float = 18.0 / 1433.0) -> GraphBatch:
    """G graphs of n nodes and e directed edges each; src, dst iid uniform in [0, n) + offset.

    SURVEY.md §8(d) "Uniform per-graph". Self-loops and duplicate edges are kept (the reference's
    `add_remaining_self_loops` removes the self-loops, `models/utils.py:58-63`)."""
    G, n, e = num_graphs, nodes_per_graph, edges_per_graph
    offs = (np.arange(G, dtype=np.int64) * n)
    gid = np.repeat(np.arange(G, dtype=np.int64), e)
    src = randint(graph_seed, G * e, n) + offs[gid]
    dst = randint(graph_seed ^ 0xD1B54A32D192ED03, G * e, n) + offs[gid]
    edge_index = np.stack([src, dst])
    N = G * n
    if features == "normal":
        x = normal(feature_seed, N * in_features).reshape(N, in_features)
    elif features == "bernoulli":
        x = (uniform01(feature_seed, N * in_features) < np.float32(bernoulli_p)).astype(np.float32)
        x = x.reshape(N, in_features)
    else:
        raise ValueError(features)
    return GraphBatch(x=x, edge_index=edge_index, num_graphs=G,
                      node_offsets=np.arange(G + 1, dtype=np.int64) * n)


def _rmat_draw(seed: int, n: int, scale: int, abcd):
    """n raw R-MAT (src, dst) pairs on a 2^scale grid (Graph500 recursive quadrant choice)."""
    a, b, c, _ = abcd
    src = np.zeros(n, dtype=np.int64)
    dst = np.zeros(n, dtype=np.int64)
    for lvl in range(scale):
        u = uniform01(seed + 1000 * (lvl + 1), n)
        right = (u >= a) & ((u < a + b) | (u >= a + b + c))   # quadrants b or d
        down = u >= a + b                                    # quadrants c or d
        src |= down.astype(np.int64) << lvl
        dst |= right.astype(np.int64) << lvl
    return src, dst


def rmat_edges(num_nodes: int, num_edges: int, seed: int = 42,
               abcd=(0.57, 0.19, 0.19, 0.05)) -> np.ndarray:
    """Graph500 R-MAT edge list (2, num_edges) int64: ids drawn on a 2^scale grid, pairs with an
    id >= num_nodes redrawn (fresh rounds of draws until exactly num_edges pairs remain), then
    vertex ids randomly permuted (SURVEY.md §8(d) "RMAT")."""
    scale = int(np.ceil(np.log2(max(num_nodes, 2))))
    srcs, dsts, have, rnd = [], [], 0, 0
    while have < num_edges:
        need = num_edges - have
        # oversample by the observed rejection rate so few rounds are needed
        n = need if rnd == 0 else int(need * 1.3) + 64
        src, dst = _rmat_draw(seed + 7919 * rnd, n, scale, abcd)
        keep = (src < num_nodes) & (dst < num_nodes)
        src, dst = src[keep][:need], dst[keep][:need]
        srcs.append(src)
        dsts.append(dst)
        have += src.size
        rnd += 1
    src, dst = np.concatenate(srcs), np.concatenate(dsts)
    perm = np.argsort(splitmix64(seed ^ 0xA5A5A5A5, num_nodes), kind="stable")
    return np.stack([perm[src], perm[dst]])


def rmat_edges_device(num_nodes: int, num_edges: int, seed: int = 42, device="cuda",
                      abcd=(0.57, 0.19, 0.19, 0.05)):
    """rmat_edges on the device with torch's generator (same R-MAT recipe, including the redraw
    of rejected pairs, not the same draws): the full-size config (1e7 nodes, exactly 1.6e8
    edges) in about a second. Returns a (2, num_edges) int64 device tensor."""
    import torch
    scale = int(np.ceil(np.log2(max(num_nodes, 2))))
    a, b, c, _ = abcd
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    srcs, dsts, have, rnd = [], [], 0, 0
    while have < num_edges:
        need = num_edges - have
        n = need if rnd == 0 else int(need * 1.3) + 64
        src = torch.zeros(n, dtype=torch.int64, device=device)
        dst = torch.zeros(n, dtype=torch.int64, device=device)
        for lvl in range(scale):
            u = torch.rand(n, generator=g, device=device)
            right = (u >= a) & ((u < a + b) | (u >= a + b + c))
            down = u >= a + b
            src |= down.to(torch.int64) << lvl
            dst |= right.to(torch.int64) << lvl
            del u, right, down
        keep = (src < num_nodes) & (dst < num_nodes)
        src, dst = src[keep][:need], dst[keep][:need]
        srcs.append(src)
        dsts.append(dst)
        have += int(src.numel())
        rnd += 1
    src = torch.cat(srcs) if len(srcs) > 1 else srcs[0]
    dst = torch.cat(dsts) if len(dsts) > 1 else dsts[0]
    del srcs, dsts
    perm = torch.randperm(num_nodes, generator=g, device=device)
    return torch.stack([perm[src], perm[dst]])


# Dataset-average shapes (SURVEY.md §8 notation block).
SHAPES = {
    "Cora": dict(nodes=2708, edges=10556, in_features=1433, features="bernoulli"),
    "PPI": dict(nodes=2245, edges=61318, in_features=50, features="normal"),
    "PATTERN": dict(nodes=119, edges=6099, in_features=3, features="normal"),
    "Citeseer": dict(nodes=3327, edges=9104, in_features=3703, features="bernoulli"),
    "Pubmed": dict(nodes=19717, edges=88648, in_features=500, features="normal"),
}


def dataset_batch(name: str, num_graphs: int = 1, graph_seed: int = 42,
                  feature_seed: int = 1) -> GraphBatch:
    s = SHAPES[name]
    return uniform_graph_batch(num_graphs, s["nodes"], s["edges"], s["in_features"],
                               graph_seed=graph_seed, feature_seed=feature_seed,
                               features=s["features"])
