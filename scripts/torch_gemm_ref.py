"""Library reference for the tower's GEMM shapes (torch.matmul -> hipBLASLt/rocBLAS), fp32."""
import torch
B = 65536
x = torch.randn(B, 416, device="cuda"); w = torch.randn(416, 400, device="cuda"); dh = torch.randn(B, 400, device="cuda")
torch.backends.cuda.matmul.allow_tf32 = False
cases = {"fwd": lambda: x @ w, "dx": lambda: dh @ w.t(), "dw": lambda: x.t() @ dh}
flops = {"fwd": 2 * B * 416 * 400, "dx": 2 * B * 400 * 416, "dw": 2 * B * 416 * 400}
for n, f in cases.items():
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print("%-4s %8.1f us %7.1f TF/s" % (n, us, flops[n] / us / 1e6))
