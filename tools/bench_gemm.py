"""GEMM microbenchmark on the box: gatx fp32 MFMA GEMM (both tile shapes) vs torch.mm (hipBLASLt)
on the PPI layer shapes (forward projection, backward g_x / g_W)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx._lib import call, ptr, stream  # noqa: E402
import ctypes  # noqa: E402
from gatx import _lib  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda:0")


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


N = 44900
shapes = [("fwd L1 x.W_aug^T", N, 1032, 1024, "nt"), ("fwd L2", N, 756, 1024, "nt"),
          ("bwd g_x = G.W_aug", N, 1024, 1032, "nn"), ("bwd g_W = G^T.x", 1032, 1024, N, "tn"),
          ("fwd L1 no-score", N, 1024, 1024, "nt")]
for name, M, Nc, K, lay in shapes:
    A = torch.randn(M, K, device=dev) if lay != "tn" else torch.randn(K, M, device=dev)
    B = torch.randn(Nc, K, device=dev) if lay == "nt" else torch.randn(K, Nc, device=dev)
    C = torch.empty(M, Nc, device=dev)
    flops = 2.0 * M * Nc * K
    if lay == "nt":
        args = (M, Nc, K, ptr(A), K, 1, ptr(B), 1, K)
        ref = lambda: torch.mm(A, B.t())
    elif lay == "nn":
        args = (M, Nc, K, ptr(A), K, 1, ptr(B), Nc, 1)
        ref = lambda: torch.mm(A, B)
    else:
        args = (M, Nc, K, ptr(A), 1, M, ptr(B), Nc, 1)
        ref = lambda: torch.mm(A.t(), B)
    res = []
    for mode in ("tail", "plain"):
        wb = _lib.lib.gatx_gemm_workspace_bytes(M, Nc, K) if mode == "tail" else 0
        wt = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
        wp = ptr(wt) if wb else None
        f = lambda: call("gatx_gemm_f32", *args, ptr(C), Nc, Nc, None, 0, 0, wp, wb, stream())
        t = timeit(f)
        err = (C - ref()).abs().max().item()
        res.append(f"{mode} {t*1e3:8.1f}us {flops/t/1e9:6.1f}TF err={err:.1e}")
    if lay == "tn":
        wsb = _lib.lib.gatx_gemm_splitk_workspace_bytes(M, Nc, K)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        f = lambda: call("gatx_gemm_f32_splitk", *args, ptr(C), Nc, 0, ptr(ws), wsb, stream())
        t = timeit(f)
        err = (C - ref()).abs().max().item()
        res.append(f"splitk {t*1e3:8.1f}us {flops/t/1e9:6.1f}TF err={err:.1e}")
    t = timeit(ref)
    res.append(f"torch.mm {t*1e3:8.1f}us {flops/t/1e9:6.1f}TF")
    print(f"{name:24s} " + " | ".join(res), flush=True)
