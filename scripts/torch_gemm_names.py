"""Run hipBLASLt (torch.matmul) on the FFN GEMM shapes so a kernel trace records which kernels it picks."""
import torch

T, D, F = 8192, 4096, 16384
bf = torch.bfloat16
x = torch.randn(T, D, device="cuda", dtype=bf)
w1 = torch.randn(F, D, device="cuda", dtype=bf)
w2 = torch.randn(D, F, device="cuda", dtype=bf)
h = torch.randn(T, F, device="cuda", dtype=bf)
dy = torch.randn(T, D, device="cuda", dtype=bf)
for _ in range(3):
    x @ w1.t()          # fwd1 NT
    h @ w2.t()          # fwd2 NT
    dy @ w2             # da NN
    h @ w1              # dx NN
    dy.t() @ h          # dW2 TN
    h.t() @ x           # dW1 TN
torch.cuda.synchronize()
