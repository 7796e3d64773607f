"""gatx_graph_segments (csrc/graph.hip, round 5): the node range cut into contiguous blocks that no
edge crosses, packed greedily up to max_rows nodes — against a numpy restatement of the same
definition on the CSR of edge_index' (self-loops rewritten as the reference does,
`models/utils.py:47-67`)."""
import numpy as np
import pytest
import torch

from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu


def _expected(ei2: np.ndarray, N: int, max_rows: int, seg_max: int = 4096):
    s, d = ei2
    lo = np.arange(N)
    hi = np.arange(N)
    np.minimum.at(lo, d, s)
    np.maximum.at(hi, d, s)
    pmax = np.maximum.accumulate(hi)                  # max hi over [0, b]
    smin = np.minimum.accumulate(lo[::-1])[::-1]      # min lo over [b, N)
    free = [b for b in range(1, N) if pmax[b - 1] < b and smin[b] >= b]
    if len(free) > seg_max:
        return None
    bnd = [0] + free + [N]
    segs, start = [0], 0
    for i in range(1, len(bnd)):
        if bnd[i] - bnd[i - 1] > max_rows:
            return None
        if bnd[i] - start > max_rows:
            segs.append(bnd[i - 1])
            start = bnd[i - 1]
    segs.append(N)
    return segs


def _blocks(device, ei, N, max_rows):
    import gatx
    from gatx.graph import graph_cache
    gatx.clear_graph_cache()
    g = graph_cache.get(torch.from_numpy(ei).to(device), N, True)
    segs, count = g.node_blocks(max_rows)
    c = int(count.item())
    return None if c < 0 else segs[:c + 1].cpu().tolist()


@pytest.mark.parametrize("case", ["ppi20", "pattern8", "pattern8_small_blocks", "isolated",
                                  "one_component", "ragged"])
def test_node_blocks_match_restatement(case, device):
    from gatx import data as gd
    if case == "ppi20":
        b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
        ei, N, R = b.edge_index, b.num_nodes, 2304
    elif case.startswith("pattern8"):
        b = gd.dataset_batch("PATTERN", 8, graph_seed=3, feature_seed=1)
        ei, N, R = b.edge_index, b.num_nodes, (2304 if case == "pattern8" else 300)
    elif case == "isolated":   # trailing isolated nodes: each its own run, packed
        ei = np.stack([gd.randint(40, 300, 50), gd.randint(41, 300, 50)])
        N, R = 60, 2304
    elif case == "one_component":   # a random graph over 3000 nodes: no block fits 2304 rows
        ei = np.stack([gd.randint(42, 30000, 3000), gd.randint(43, 30000, 3000)])
        N, R = 3000, 2304
    else:   # graphs of ragged sizes, some larger than max_rows / 2
        sizes = [700, 1500, 30, 2000, 1, 900, 1200]
        parts, off = [], 0
        for i, n in enumerate(sizes):
            e = 8 * n
            parts.append(np.stack([gd.randint(50 + i, e, n), gd.randint(60 + i, e, n)]) + off)
            off += n
        ei, N, R = np.concatenate(parts, axis=1), off, 2304
    ei2 = orc.add_remaining_self_loops(ei, N)
    want = _expected(ei2, N, R)
    got = _blocks(device, ei, N, R)
    assert got == want, (case, got[:8] if got else got, want[:8] if want else want)
    if case == "ppi20":
        assert got == [2245 * k for k in range(21)]
    if case == "pattern8":
        assert got == [0, N]
    if case == "one_component":
        assert got is None
