"""Concurrency probe: the PPI layer-1 projection GEMM and a layer-1 edge pass (independent data)
on two HIP streams at once vs back to back, for GEMM variants GATX_GEMM_BK (set per run)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx._lib import ARGMAX_CAP, call, lib, ptr  # noqa: E402
from gatx.graph import Graph  # noqa: E402

dev = torch.device("cuda:0")
b = gd.dataset_batch("PPI", 20)
N = b.num_nodes
g = Graph(torch.from_numpy(b.edge_index).to(dev), N, True)
E2 = g.num_edges
NH, F, Fp = 4, 256, 256
x = torch.randn(N, 1024, device=dev)
W = torch.randn(1024, 1024, device=dev)
C = torch.empty(N, 1024, device=dev)
wb = lib.gatx_gemm_workspace_bytes(N, 1024, 1024)
ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
Wh = torch.randn(N, NH * Fp, device=dev)
S = torch.randn(N, 2 * NH, device=dev)
M = torch.zeros(1, dtype=torch.int32, device=dev)
mws = torch.empty(lib.gatx_attention_max_workspace_bytes(), dtype=torch.uint8, device=dev)
call("gatx_attention_max", ptr(g.col), ptr(g.rowidx), E2, ptr(S), NH, ptr(M), None, ptr(mws),
     torch.cuda.current_stream().cuda_stream)
out = torch.empty(N, NH * F, device=dev)
den = torch.empty(N, NH, device=dev)
sA = torch.cuda.Stream()
sB = torch.cuda.Stream()


def gemm(s):
    call("gatx_projection_gemm", N, 1024, 1024, ptr(x), 1024, 1, ptr(W), 1, 1024, ptr(C), 1024,
         1024, None, 0, ptr(ws) if wb else None, wb, s.cuda_stream)


def edge(s):
    call("gatx_edge_forward_ex", ptr(Wh), NH * Fp, Fp, ptr(S), ptr(M), ptr(g.rowptr), ptr(g.col),
         ptr(g.perm), N, NH, F, 1, 1, 0, None, 0.0, 0, ptr(out), NH * F, None, 0, 0, ptr(den),
         2048, s.cuda_stream)


def timed(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def seq():
    gemm(torch.cuda.current_stream()); edge(torch.cuda.current_stream())


def par():
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event(); ev.record(cur)
    sA.wait_event(ev); sB.wait_event(ev)
    gemm(sA); edge(sB)
    ea = torch.cuda.Event(); ea.record(sA); eb = torch.cuda.Event(); eb.record(sB)
    cur.wait_event(ea); cur.wait_event(eb)


def par_half():   # edge on half the rows, started alongside the gemm
    par()


print(f"BK={os.environ.get('GATX_GEMM_BK', '17')} gemm alone {timed(lambda: gemm(torch.cuda.current_stream())):7.1f} us | "
      f"edge alone {timed(lambda: edge(torch.cuda.current_stream())):7.1f} us | "
      f"sequential {timed(seq):7.1f} us | concurrent {timed(par):7.1f} us", flush=True)
