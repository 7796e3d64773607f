"""Host-side cost of one per-step graph build (PPI bench batch): total Graph() construction with
the GPU idle, the stats read-back alone, and the host time of a whole forward step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx.graph import Graph  # noqa: E402
from gatx._lib import call, ptr, stream, lib  # noqa: E402

dev = torch.device("cuda:0")
b = gd.uniform_graph_batch(20, 2245, 61318, 50)
ei = torch.from_numpy(b.edge_index).to(dev)
for _ in range(5):
    Graph(ei, b.num_nodes, True)
torch.cuda.synchronize()
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Graph(ei, b.num_nodes, True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t.append((t1 - t0) * 1e6)
print(f"Graph() host time (GPU idle at entry): median {sorted(t)[10]:.1f} us")
stats = torch.empty(3, dtype=torch.int64, device=dev)
sws = torch.empty(lib.gatx_edge_stats_workspace_bytes(), dtype=torch.uint8, device=dev)
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call("gatx_edge_stats", ptr(ei), 1, ei.size(1), ei.stride(0), ptr(stats), ptr(sws), stream())
    v = stats.cpu()
    t1 = time.perf_counter()
    t.append((t1 - t0) * 1e6)
print(f"stats launch + .cpu(): median {sorted(t)[10]:.1f} us")
pin = torch.empty(3, dtype=torch.int64, pin_memory=True)
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call("gatx_edge_stats", ptr(ei), 1, ei.size(1), ei.stride(0), ptr(stats), ptr(sws), stream())
    pin.copy_(stats, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    v = pin.tolist()
    t1 = time.perf_counter()
    t.append((t1 - t0) * 1e6)
print(f"stats launch + pinned copy + sync: median {sorted(t)[10]:.1f} us")
t = []
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    E2 = 1270712
    i32 = dict(dtype=torch.int32, device=dev)
    a = [torch.empty(44901, **i32)] + [torch.empty(E2, **i32) for _ in range(3)]
    e2 = torch.empty((2, E2), dtype=torch.int64, device=dev)
    wsb = lib.gatx_graph_build_workspace_bytes(ei.size(1), E2, 44900)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    t1 = time.perf_counter()
    t.append((t1 - t0) * 1e6)
print(f"allocations + workspace query: median {sorted(t)[10]:.1f} us")
# phases of Graph.__init__ after the sync (host only)
E = ei.size(1)
E2 = 1270712
N = 44900
i32 = dict(dtype=torch.int32, device=dev)
rowptr = torch.empty(N + 1, **i32); col = torch.empty(E2, **i32); rowidx = torch.empty(E2, **i32)
perm = torch.empty(E2, **i32); e2 = torch.empty((2, E2), dtype=torch.int64, device=dev)
res = {"wsq": [], "alloc_ws": [], "build_call": []}
for _ in range(20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wsb = lib.gatx_graph_build_workspace_bytes(E, E2, N)
    t1 = time.perf_counter()
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    t2 = time.perf_counter()
    call("gatx_graph_build", ptr(ei), 1, E, ei.stride(0), 1, N, N, E2, ptr(e2), ptr(rowptr),
         ptr(col), ptr(rowidx), ptr(perm), ptr(ws), wsb, stream())
    t3 = time.perf_counter()
    res["wsq"].append((t1 - t0) * 1e6); res["alloc_ws"].append((t2 - t1) * 1e6)
    res["build_call"].append((t3 - t2) * 1e6)
for k, v in res.items():
    print(f"{k}: median {sorted(v)[10]:.1f} us")
