"""torch.mm (hipBLASLt) on the PPI GEMM shapes, for reading the chosen Tensile kernels in a trace."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda:0")
N = 44900
for (M, Nc, K, lay) in [(N, 1024, 1024, "nt"), (N, 756, 1024, "nt"), (N, 1024, 1032, "nn")]:
    A = torch.randn(M, K, device=dev)
    B = torch.randn(Nc, K, device=dev) if lay == "nt" else torch.randn(K, Nc, device=dev)
    for _ in range(3):
        C = A @ (B.t() if lay == "nt" else B)
torch.cuda.synchronize()
print("ok")
