"""Times the C5 bf16 tower's GEMM shapes through the C ABI (HIP events).
python scripts/gemm_bf16_bench.py [reps] [case substring]"""
import sys

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 else None   # run the cases whose names contain this (profiling)
B = 65536
s = _lib.stream_handle()
bf = lambda *sh: torch.randn(*sh, device="cuda").to(torch.bfloat16)
x0 = bf(B, 432)
h = bf(B, 416)
hT = bf(416, B)
dhT = bf(416, B)
WT = bf(400, 432)          # W^T, k-contiguous
W1 = bf(416, 400)
out_b = torch.zeros(B, 416, device="cuda", dtype=torch.bfloat16)
out_f = torch.zeros(B, 416, device="cuda")
slab = torch.zeros(96 * 432 * 416, device="cuda")
u16 = lambda t: ptr(t)
cases = {
    "fwd_l0 bf16 out relu": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 432, u16(x0), 432, u16(WT), 432, ptr(out_b), 416, 1, 1,
                                          None, 0, 1, 0, s), 2 * B * 433 * 400),
    "fwd_l0 f32 out": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 432, u16(x0), 432, u16(WT), 432, ptr(out_f), 416, 0, 0,
                                    None, 0, 1, 0, s), 2 * B * 433 * 400),
    "dx_l1 mask bf16": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 400, u16(h), 416, u16(W1), 400, ptr(out_b), 416, 1, 2,
                                     u16(h), 416, 1, 0, s), 2 * B * 400 * 400),
    "dw_l1 split64": (lambda: call("dl_gemm_bf16", 0, 1, 416, 400, B, u16(hT), B, u16(dhT), B, ptr(slab), 400, 0, 3, None, 0,
                                   64, 416 * 400, s), 2 * B * 417 * 400),
    "dw_l1 direct (ta=1) split64": (lambda: call("dl_gemm_bf16", 1, 0, 416, 400, B, u16(h), 416, u16(out_b), 416,
                                                 ptr(slab), 400, 0, 3, None, 0, 64, 416 * 400, s), 2 * B * 417 * 400),
    "dw_l0 direct (ta=1) split85": (lambda: call("dl_gemm_bf16", 1, 0, 432, 400, B, u16(x0), 432, u16(out_b), 416,
                                                 ptr(slab), 400, 0, 3, None, 0, 85, 432 * 400, s), 2 * B * 433 * 400),
    "dw_l1 direct (ta=1) split85": (lambda: call("dl_gemm_bf16", 1, 0, 416, 400, B, u16(h), 416, u16(out_b), 416,
                                                 ptr(slab), 400, 0, 3, None, 0, 85, 416 * 400, s), 2 * B * 417 * 400),
    "transpose_bf16 [B,416]": (lambda: call("dl_transpose_bf16", u16(h), 0, B, 416, 416, u16(hT), B, s), 0),
    "cast_bf16 [B,416]": (lambda: call("dl_cast_bf16", ptr(out_f), B, 416, 416, u16(out_b), 416, s), 0),
}
for name, (fn, fl) in cases.items():
    if only and only not in name:
        continue
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
    print("%-26s %8.1f us  %7.1f TF/s" % (name, us, fl / us / 1e6 if fl else 0.0), flush=True)
