"""One GEMM shape, repeated (for rocprofv3 PMC passes): python tools/gemm_one.py MODE LAYOUT M N K [reps]
MODE 0 = f32 MFMA, 1 = split-bf16 x3; LAYOUT nt|nn|tn|tt (A then B: n = k-contiguous)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx._lib import call, ptr, stream, lib  # noqa: E402

mode, lay = int(sys.argv[1]), sys.argv[2]
M, Nc, K = (int(v) for v in sys.argv[3:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda:0")
A = torch.randn(M, K, device=dev) if lay[0] == "n" else torch.randn(K, M, device=dev)
B = torch.randn(Nc, K, device=dev) if lay[1] == "t" else torch.randn(K, Nc, device=dev)
C = torch.empty(M, Nc, device=dev)
sam, sak = (K, 1) if lay[0] == "n" else (1, M)
sbk, sbn = (1, K) if lay[1] == "t" else (Nc, 1)
lib.gatx_set_gemm_mode(mode)
wb = lib.gatx_gemm_workspace_bytes(M, Nc, K)
wt = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
for i in range(reps + 1):
    if i == 1:
        s.record()
    call("gatx_gemm_f32", M, Nc, K, ptr(A), sam, sak, ptr(B), sbk, sbn, ptr(C), Nc, Nc, None, 0, 0,
         ptr(wt) if wb else None, wb, stream())
e.record(); torch.cuda.synchronize()
t = s.elapsed_time(e) / reps
print(f"mode {mode} {lay} {M}x{Nc}x{K}: {t*1e3:.1f} us {2.0*M*Nc*K/t/1e9:.1f} TF")
if os.environ.get("GEMM_CHECK"):
    torch.backends.cuda.matmul.allow_tf32 = False
    Am = A if lay[0] == "n" else A.t()
    Bm = B.t() if lay[1] == "t" else B
    ref = (Am[:512].double() @ Bm.double())
    err = ((C[:512].double() - ref).abs().max() / ref.abs().max()).item()
    print(f"  check rows 0-511: max rel err {err:.2e}")
