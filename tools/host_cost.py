"""Host cost per call (steady state, no sync inside the loop) of torch F.linear on PATTERN's skip
shapes vs gatx_gemm_f32 through ctypes, and of an empty gatx launch path."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
import torch.nn.functional as Fn  # noqa: E402
from gatx._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
N = 3808
for fin, fout in [(3, 48), (48, 96), (96, 48), (48, 1)]:
    x = torch.randn(N, fin, device=dev)
    W = torch.randn(fout, fin, device=dev)
    C = torch.empty(N, fout, device=dev)
    for _ in range(20):
        Fn.linear(x, W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        Fn.linear(x, W)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(500):
        call("gatx_gemm_f32", N, fout, fin, ptr(x), fin, 1, ptr(W), 1, fin, ptr(C), fout, fout,
             None, 0, 0, None, 0, stream())
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{fin:3d}->{fout:3d}: F.linear host {1e6 * (t1 - t0) / 500:6.1f} us/call | "
          f"gatx_gemm_f32 host {1e6 * (t3 - t2) / 500:6.1f} us/call", flush=True)
