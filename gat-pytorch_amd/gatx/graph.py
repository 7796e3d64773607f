"""Device-side graph preprocessing for the GAT layer: the self-loop rewrite + destination CSR
(and, for the backward, the source-ordered transpose), cached per edge_index.

The reference rewrites self-loops inside every forward of every layer
(`models/gat_layer.py:53-54` -> `models/utils.py:47-67`) and then scatters/gathers by raw edge
indices. Here the rewrite and the CSR build run once per distinct edge_index on the GPU
(`gatx_edge_stats` + `gatx_graph_build`, csrc/graph.hip) and are reused by every layer and step
that sees the same tensor. The one host sync per new graph is the reference's own
`int(index.max())` (`models/utils.py:70-72`), which sizes edge_index'.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from . import _lib
from ._lib import call, ptr, stream, version


class Graph:
    """CSR of edge_index' (int32), plus the returned edge_index' tensor itself.

    rowptr [N+1], col [E2] (source), rowidx [E2] (destination), perm [E2] (CSR slot -> position
    in edge_index'); srowptr / scol / seid: the source-ordered transpose, built on first use."""

    def __init__(self, edge_index: torch.Tensor, num_nodes, add_self_loops: bool):
        """num_nodes None: size the node range from the edges (max id + 1)."""
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise RuntimeError(f"edge_index must have shape (2, E), got {tuple(edge_index.shape)}")
        if edge_index.dtype not in (torch.int64, torch.int32):
            raise RuntimeError(f"edge_index must be int64 or int32, got {edge_index.dtype}")
        if not edge_index.is_cuda:
            raise RuntimeError("gatx: edge_index must be on the HIP device (no CPU path)")
        dev = edge_index.device
        if edge_index.stride(1) != 1:
            edge_index = edge_index.contiguous()
        self.device = dev
        self.add_self_loops = add_self_loops
        E = edge_index.size(1)
        is64 = int(edge_index.dtype == torch.int64)
        ld = edge_index.stride(0)
        if E == 0 and add_self_loops:
            # maybe_num_nodes: int(index.max()) on an empty tensor (models/utils.py:72)
            raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0. "
                               "Specify the reduction dim with the 'dim' argument.")
        s = stream()
        stats = torch.empty(3, dtype=torch.int64, device=dev)
        sws = torch.empty(_lib.lib.gatx_edge_stats_workspace_bytes(), dtype=torch.uint8,
                          device=dev)
        call("gatx_edge_stats", ptr(edge_index), is64, E, ld, ptr(stats), ptr(sws), s)
        mn, mx, nloops = (int(v) for v in stats.cpu())   # the one host sync per new graph
        if num_nodes is None:
            num_nodes = mx + 1 if E else 0
        self.num_nodes = N = int(num_nodes)
        if E and mn < 0:
            raise RuntimeError(f"index {mn} is out of bounds: edge_index has negative node ids")
        if E and mx >= N:
            raise IndexError(f"index {mx} is out of bounds for dimension 0 with size {N}")
        if add_self_loops:
            num_loops = mx + 1
            E2 = E - nloops + num_loops
        else:
            num_loops = 0
            E2 = E
        self.num_edges = E2
        i32 = dict(dtype=torch.int32, device=dev)
        self.rowptr = torch.empty(N + 1, **i32)
        self.col = torch.empty(max(E2, 1), **i32)
        self.rowidx = torch.empty(max(E2, 1), **i32)
        self.perm = torch.empty(max(E2, 1), **i32)
        if add_self_loops:
            self.edge_index = torch.empty((2, E2), dtype=torch.int64, device=dev)
            ei_out = ptr(self.edge_index)
        else:
            self.edge_index = edge_index   # the reference returns its input unchanged
            ei_out = None
        ws_bytes = _lib.lib.gatx_graph_build_workspace_bytes(E, E2, N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        call("gatx_graph_build", ptr(edge_index), is64, E, ld, int(add_self_loops), num_loops, N,
             E2, ei_out, ptr(self.rowptr), ptr(self.col), ptr(self.rowidx), ptr(self.perm),
             ptr(ws), ws_bytes, s)
        self.srowptr = self.scol = self.seid = None

    def ensure_transpose(self):
        if self.srowptr is not None:
            return
        N, E2, dev = self.num_nodes, self.num_edges, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.srowptr = torch.empty(N + 1, **i32)
        self.scol = torch.empty(max(E2, 1), **i32)
        self.seid = torch.empty(max(E2, 1), **i32)
        ws_bytes = _lib.lib.gatx_graph_transpose_workspace_bytes(E2, N)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        call("gatx_graph_transpose", ptr(self.col), ptr(self.rowidx), N, E2, ptr(self.srowptr),
             ptr(self.scol), ptr(self.seid), ptr(ws), ws_bytes, stream())

    def csr_host(self):
        """(rowptr, col, perm) as CPU tensors — for tests."""
        E2 = self.num_edges
        return self.rowptr.cpu(), self.col[:E2].cpu(), self.perm[:E2].cpu()


class GraphCache:
    """Small LRU of Graphs keyed on the edge_index tensor's identity and version. Entries hold a
    reference to their key tensor, so a cached data_ptr can never be recycled under them. A
    Graph built with add_self_loops also answers for its own output edge_index' (the rewrite is
    idempotent, so GATModel.forward_and_return_attention's chaining of layers hits the cache)."""

    def __init__(self, capacity: int = 8):
        self.capacity = capacity
        self._d: OrderedDict = OrderedDict()

    @staticmethod
    def _key(t: torch.Tensor, num_nodes: int, add_self_loops: bool):
        return (t.data_ptr(), version(t), tuple(t.shape), tuple(t.stride()), t.dtype,
                t.device, num_nodes, add_self_loops)

    def get(self, edge_index: torch.Tensor, num_nodes: int, add_self_loops: bool) -> Graph:
        k = self._key(edge_index, num_nodes, add_self_loops)
        hit = self._d.get(k)
        if hit is not None:
            self._d.move_to_end(k)
            return hit[1]
        g = Graph(edge_index, num_nodes, add_self_loops)
        self._put(k, edge_index, g)
        if add_self_loops:
            self._put(self._key(g.edge_index, num_nodes, True), g.edge_index, g)
        return g

    def for_edges(self, edge_index: torch.Tensor) -> Graph:
        """The Graph whose edge_index' IS this tensor (what a layer returned), else a CSR of it
        as given (no rewrite), sized by its max id — for consumers of a layer's output edges
        such as the attention-norm regulariser."""
        for t, g in reversed(self._d.values()):
            ei = g.edge_index
            if ei is edge_index or (ei.data_ptr() == edge_index.data_ptr()
                                    and version(ei) == version(edge_index)
                                    and ei.shape == edge_index.shape
                                    and ei.stride() == edge_index.stride()
                                    and ei.dtype == edge_index.dtype):
                return g
        k = self._key(edge_index, -1, False)
        hit = self._d.get(k)
        if hit is not None:
            return hit[1]
        g = Graph(edge_index, None, False)
        self._put(k, edge_index, g)
        return g

    def _put(self, k, t, g):
        self._d[k] = (t, g)
        self._d.move_to_end(k)
        while len(self._d) > self.capacity:
            self._d.popitem(last=False)

    def clear(self):
        self._d.clear()


graph_cache = GraphCache()


def clear_graph_cache():
    graph_cache.clear()
