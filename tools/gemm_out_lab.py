"""gemm_out (PPI layer 0 per-head output projection) in isolation: batched GEMM with and
without the ELU / bias epilogue, and as 4 separate GEMMs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
N, NH, F, FIN, FP = 44900, 4, 256, 50, 52


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


Z = torch.randn(N, NH * FP, device=dev)
Wp = torch.randn(NH * F, FP, device=dev)
out = torch.empty(N, NH * F, device=dev)
for elu in (0, 1):
    f = lambda: call("gatx_gemm_f32_batched", NH, N, F, FIN, ptr(Z), NH * FP, 1, FP, ptr(Wp), 1,
                     FP, F * FP, ptr(out), NH * F, F, 0, None, F, None, NH * F, F, elu, stream())
    print(f"batched elu={elu}: {timeit(f):7.1f} us", flush=True)
f = lambda: [call("gatx_gemm_f32_batched", 1, N, F, FIN, ptr(Z) + 4 * h * FP, NH * FP, 1, 0,
                  ptr(Wp) + 4 * h * F * FP, 1, FP, 0, ptr(out) + 4 * h * F, NH * F, 0, 0, None, 0,
                  None, NH * F, 0, 0, stream()) for h in range(NH)]
print(f"4 separate: {timeit(f):7.1f} us", flush=True)
f = lambda: out.copy_(out)
print(f"out.copy_ (read+write 184 MB): {timeit(f):7.1f} us", flush=True)
f = lambda: out.zero_()
print(f"out.zero_ (write 184 MB): {timeit(f):7.1f} us", flush=True)
