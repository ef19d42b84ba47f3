"""Times the C2 tower's GEMM shapes through the C ABI (HIP events), for tuning and
for rocprofv3 PMC passes:  python scripts/gemm_bench.py [reps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = 65536
s = _lib.stream_handle()
z = lambda *sh: torch.randn(*sh, device="cuda")
x0, h, dh = z(B, 432), z(B, 416), z(B, 416)
W0, W1, Wt = z(432, 400), z(416, 400), z(400, 432)
slab = torch.zeros(64 * 432 * 400, device="cuda")
cases = {
    "fwd_l0": lambda: call("dl_gemm_f32", 0, 0, B, 400, 432, ptr(x0), 432, ptr(W0), 400, ptr(h), 416, 1, None, 0, 1, 0, s),
    "fwd_l1": lambda: call("dl_gemm_f32", 0, 0, B, 400, 416, ptr(h), 416, ptr(W1), 400, ptr(dh), 416, 1, None, 0, 1, 0, s),
    "dx_l1": lambda: call("dl_gemm_f32", 0, 0, B, 400, 400, ptr(dh), 416, ptr(Wt), 432, ptr(h), 416, 2, ptr(x0), 432, 1, 0, s),
    "dw_l1": lambda: call("dl_gemm_f32", 1, 0, 416, 400, B, ptr(h), 416, ptr(dh), 416, ptr(slab), 400, 3, None, 0, 64,
                          416 * 400, s),
    "dw_l0": lambda: call("dl_gemm_f32", 1, 0, 432, 400, B, ptr(x0), 432, ptr(dh), 416, ptr(slab), 400, 3, None, 0, 64,
                          432 * 400, s),
}
flops = {"fwd_l0": 2 * B * 433 * 400, "fwd_l1": 2 * B * 417 * 400, "dx_l1": 2 * B * 400 * 400, "dw_l1": 2 * B * 417 * 400, "dw_l0": 2 * B * 433 * 400}
for name, fn in cases.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print("%-7s %8.1f us  %6.1f TF/s" % (name, us, flops[name] / us / 1e6), flush=True)

# split-K sweep of the dW product (layer 1 shape)
slab2 = torch.zeros(256 * 416 * 400, device="cuda")
for sp in (16, 32, 48, 64, 96, 128, 192, 256):
    fn = lambda: call("dl_gemm_f32", 1, 0, 416, 400, B, ptr(h), 416, ptr(dh), 416, ptr(slab2), 400, 3, None, 0, sp,
                      416 * 400, s)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print("dw_l1 splits %3d %8.1f us  %6.1f TF/s" % (sp, us, flops["dw_l1"] / us / 1e6), flush=True)
