"""wdl head cost split (C5 shape): full launch vs no wide-gradient atomics (g_w = NULL),
and with all wide ids in a small range (atomics L2-resident)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

B, Fw, H, ldh, rows = 65536, 26, 400, 404, 26_000_000 + 426
s = _lib.stream_handle()
g = torch.Generator(device="cuda").manual_seed(1)
h = torch.rand(B, ldh, device="cuda", generator=g)
w = torch.rand(rows, device="cuda", generator=g) * 0.01
bias = torch.zeros(4, device="cuda")
label = (torch.rand(B, device="cuda", generator=g) > 0.5).float()
score, z, dz = (torch.zeros(B, device="cuda") for _ in range(3))
dh = torch.zeros(B, ldh, device="cuda", dtype=torch.bfloat16)
gw = torch.zeros(rows, device="cuda")
touched = torch.zeros(rows, device="cuda", dtype=torch.uint8)
grid = _lib.lib().dl_wdl_head_grid(B)
slab = torch.zeros(grid * (H + 2), device="cuda")
err = torch.zeros(4, device="cuda", dtype=torch.int32)


def run(wide, with_grad, n=20, flags=True):
    args = lambda: (B, Fw, H, ptr(wide), Fw, ptr(h), ldh, ptr(w), ptr(bias), rows, ptr(label), 1e-7, 1.0 / B,
                    ptr(score), ptr(z), ptr(dz), ptr(dh), ptr(gw) if with_grad else None,
                    ptr(touched) if (with_grad and flags) else None, ptr(slab), grid, ptr(err), s)
    for _ in range(3):
        call("dl_wdl_head_fwd_bwd_bf16", *args())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        call("dl_wdl_head_fwd_bwd_bf16", *args())
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


wide_u = torch.randint(0, 26_000_000, (B, Fw), device="cuda", generator=g)
wide_s = torch.randint(0, 65536, (B, Fw), device="cuda", generator=g)
print("uniform ids, full          %.1f us" % run(wide_u, True))
print("uniform ids, no grad/flags %.1f us" % run(wide_u, False))
print("uniform ids, grad no flags %.1f us" % run(wide_u, True, flags=False))
print("64K-row ids, full          %.1f us" % run(wide_s, True))
print("64K-row ids, no grad/flags %.1f us" % run(wide_s, False))
