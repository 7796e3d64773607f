"""Edge-pass laboratory (GPU box): times gatx_edge_forward_ex on the PPI G=20 layer-1 / layer-2
shapes under different work-item shapes and diagnostic ablations (gatx_set_debug)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx._lib import ARGMAX_CAP, call, lib, ptr, stream  # noqa: E402
from gatx.graph import Graph  # noqa: E402

dev = torch.device("cuda:0")
G = int(os.environ.get("G", "20"))
b = gd.dataset_batch("PPI", G)
N = b.num_nodes
g = Graph(torch.from_numpy(b.edge_index).to(dev), N, True)
E2 = g.num_edges


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for (NH, F, concat) in [(4, 256, 1), (6, 121, 0), (6, 121, 1)]:
    Fp = (F + 3) // 4 * 4
    Wh = torch.randn(N, NH * Fp, device=dev)
    S = torch.randn(N, 2 * NH, device=dev)
    M = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(lib.gatx_attention_max_workspace_bytes(), dtype=torch.uint8, device=dev)
    call("gatx_attention_max", ptr(g.col), ptr(g.rowidx), E2, ptr(S), NH, ptr(M), None, ptr(ws), stream())
    out = torch.empty(N, NH * F if concat else F, device=dev)
    alpha = torch.empty(E2, NH, device=dev)
    den = torch.empty(N, NH, device=dev)
    am = torch.zeros(ARGMAX_CAP + 2, dtype=torch.int64, device=dev)
    alg = 4.0 * E2 * NH * F
    for hs in ([d for d in (1, 2, 3, 4, 6) if NH % d == 0] if concat else [NH]):
        for chunk in ([1024, 2048, 4096] if hs <= 2 else [2048]):
            for dbg in (0,):
                lib.gatx_set_debug(dbg)
                f = lambda: call("gatx_edge_forward_ex", ptr(Wh), NH * Fp, Fp, ptr(S), ptr(M),
                                 ptr(g.rowptr), ptr(g.col), ptr(g.perm), N, NH, F, hs, concat, 0,
                                 None, 0.0, 0, ptr(out), out.size(1), None, 0, 0,
                                 ptr(den), chunk, stream())
                t = timeit(f)
                print(f"NH={NH} F={F} hs={hs} chunk={chunk:>10} dbg={dbg}: {t:8.1f} us "
                      f"({alg / t / 1e3:7.0f} GB/s alg)", flush=True)
    lib.gatx_set_debug(0)
    fa = lambda: call("gatx_attention_alpha", ptr(g.col), ptr(g.rowidx), ptr(g.perm), E2, ptr(S),
                      ptr(M), ptr(den), NH, 0, ptr(alpha), ptr(am), stream())
    print(f"NH={NH} attention_alpha: {timeit(fa):8.1f} us", flush=True)
