"""Runs one gatx GEMM shape a few times (for rocprofv3 counter passes on the box).
usage: python tools/gemm_probe.py M N K [reps] [tail]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx._lib import call, ptr, stream, lib  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
tail = len(sys.argv) > 5 and sys.argv[5] == "tail"
dev = torch.device("cuda:0")
A = torch.randn(M, K, device=dev)
B = torch.randn(N, K, device=dev)
C = torch.empty(M, N, device=dev)
wb = lib.gatx_gemm_workspace_bytes(M, N, K) if tail else 0
ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
for _ in range(reps):
    call("gatx_gemm_f32", M, N, K, ptr(A), K, 1, ptr(B), 1, K, ptr(C), N, N, None, 0, 0,
         ptr(ws) if wb else None, wb, stream())
torch.cuda.synchronize()
print("ok", (C - A @ B.t()).abs().max().item())
