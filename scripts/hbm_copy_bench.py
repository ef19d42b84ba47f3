"""The HBM streaming yardstick: dl_hbm_copy (metrics.hip) against torch's copy_ at a few sizes
(HIP events, GB/s = read + written bytes / time).  python scripts/hbm_copy_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

s = _lib.stream_handle()
for gib in (0.25, 1.0, 4.0):
    n = int(gib * (1 << 30))
    a = torch.ones(n // 4, device="cuda")
    b = torch.empty_like(a)
    for name, fn in (("dl_hbm_copy", lambda: call("dl_hbm_copy", ptr(a), ptr(b), n, s)),
                     ("torch copy_", lambda: b.copy_(a))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 10
        print("%-12s %5.2f GiB  %8.1f us  %7.1f GB/s" % (name, gib, us, 2 * n / us / 1e3), flush=True)
    del a, b
    torch.cuda.empty_cache()
