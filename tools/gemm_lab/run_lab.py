"""GEMM lab (tuning only): the f16v2 lab kernels (tools/gemm_lab/f16lab.hip) against the library's
shipped f16x3 kernel (gatx_gemm_f32 / gatx_projection_gemm) on the PPI projection shapes.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); every variant's result
checked against fp64.
    python tools/gemm_lab/run_lab.py"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402
from gatx import _lib  # noqa: E402
from gatx._lib import call, ptr, stream  # noqa: E402

lab = ctypes.CDLL(os.path.join(HERE, "libf16lab.so"))
P, I64, I, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
lab.lab_split_b.argtypes = [P, I64, I64, I64, F, P, P]
lab.lab_gemm.argtypes = [I, I, P, I64, P, I64, I64, I64, F, P, I64, P, P]
lab.lab_gemm_pp.argtypes = [I, P, P, P, I64, I64, I64, F, P, I64, P]
dev = torch.device("cuda:0")


def timed(fn, reps=10):
    fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3   # us


def main():
    shapes = [("L1 44900x1024x1024", 44900, 1024, 1024), ("L2 44900x768x1024", 44900, 768, 1024),
              ("8192^2 x 4096", 8192, 8192, 4096)]
    if os.environ.get("LAB_SHAPES") == "waves":   # the L1 shape at whole / partial waves of tiles
        shapes = [(f"M={m} ({(m + 255) // 256 * 4} tiles) x1024x1024", m, 1024, 1024)
                  for m in (32768, 40960, 44900, 49152)]
    for name, M, N, K in shapes:
        g = torch.Generator(device=dev).manual_seed(1)
        A = torch.randn(M, K, device=dev, generator=g)
        A = torch.nn.functional.elu(A)                 # activation-like rows
        B = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.054   # xavier-like weights
        ref = (A.double() @ B.double().t())
        scale = (A.abs().double() @ B.abs().double().t())
        bmax = float(B.abs().max())
        e = torch.frexp(torch.tensor(bmax)).exponent.item()
        sB = 2.0 ** (10 - e)
        Bp = torch.empty(N * K * 2, dtype=torch.uint16, device=dev)
        lab.lab_split_b(ptr(B), N, K, K, 32.0 * sB, ptr(Bp), stream())
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        C = torch.empty(M, N, device=dev)
        wsb = _lib.lib.gatx_gemm_workspace_bytes(M, N, K)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)

        def lib_run():
            call("gatx_gemm_f32", M, N, K, ptr(A), K, 1, ptr(B), 1, K, ptr(C), N, N, None, 0, 0,
                 ptr(ws) if wsb else None, wsb, stream())

        Ap = torch.empty(M * K * 2, dtype=torch.uint16, device=dev)
        lab.lab_split_b(ptr(A), M, K, K, 64.0, ptr(Ap), stream())   # A planes, Ah = fp16(64 a)
        from gatx.functional import build_weight_planes
        planes = build_weight_planes(B, N, K, K)

        def lib_planes_run():   # the library's pre-split kernel (ping-pong loop), no scores
            call("gatx_gemm_planes", M, N, K, ptr(A), K, ptr(B), K, ptr(planes), ptr(C), N, N,
                 None, 0, -1, None, 0, 0, None, 0, 0, None, 0, None, ptr(ws) if wsb else None,
                 wsb, stream())

        def pp(bk):
            return lambda: lab.lab_gemm_pp(bk, None, ptr(Ap), ptr(Bp), M, N, K, 2.0 ** -11 / sB,
                                           ptr(C), N, stream())

        def v2(bk, sc=0):
            return lambda: lab.lab_gemm(bk, sc, ptr(A), K, ptr(Bp), M, N, K, 2.0 ** -11 / sB,
                                        ptr(C), N, ptr(bad), stream())

        variants = {"lib f16x3": lib_run, "lib f16p (planes, ping-pong)": lib_planes_run,
                    "v4 A+B planes bk16": pp(16), "v5 glds ring4 bk16": pp(5),
                    "v7 ping-pong, A+B planes": pp(7), "v8 pp + glds ring (row-major), A+B planes": pp(8),
                    "v2 bk16 scale0": v2(16), "v3 16x16x32 scale0": v2(33),
                    "v6 ping-pong bk16": v2(6), "v6 + 99.5 KB LDS": v2(60),
                    "v8 pp + glds ring (row-major), A split": v2(8)}
        only = os.environ.get("LAB_ONLY")
        if only:
            variants = {k: f for k, f in variants.items() if any(t in k for t in only.split(","))}
        errs = {}
        for vn, fn in variants.items():
            C.zero_()
            bad.zero_()
            fn()
            torch.cuda.synchronize()
            errs[vn] = (float(((C.double() - ref).abs() / (scale + 1e-30)).max()), int(bad.item()))
        times = {vn: [] for vn in variants}
        for _ in range(5):
            for vn, fn in variants.items():
                times[vn].append(timed(fn))
        flop = 2.0 * M * N * K
        print(f"== {name}", flush=True)
        for vn in variants:
            t = statistics.median(times[vn])
            print(f"  {vn:22s} {t:8.1f} us  {flop / t / 1e6:7.1f} TF  (min {min(times[vn]):.1f})"
                  f"  rel.err {errs[vn][0]:.2e}  bad_tiles {errs[vn][1]}", flush=True)


if __name__ == "__main__":
    main()
