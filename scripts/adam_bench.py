"""Times the tower's dense Adam updates through the C ABI (HIP events): slab counts and the
operand-copy variants (none / bf16 copy + transpose / s3 planes).  python scripts/adam_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

s = _lib.stream_handle()
R, C = 432, 400
n = R * C
p, m, v = (torch.rand(n, device="cuda") for _ in range(3))
slab = torch.randn(96 * n, device="cuda") * 1e-3
opt = torch.zeros(_lib.OPT_LEN, device="cuda")
call("dl_adam_begin_step", ptr(opt), 0.9, 1e7, s)
wb = torch.zeros(3 * n, dtype=torch.int16, device="cuda")
wbt = torch.zeros(3 * n, dtype=torch.int16, device="cuda")


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for ns in (1, 32, 79):
    t0 = timeit(lambda: call("dl_adam_dense_reg", ptr(p), ptr(m), ptr(v), ptr(slab), ns, n, n, 0.0, 0, 0, ptr(opt),
                             None, None, s))
    t1 = timeit(lambda: call("dl_adam_dense_bf16", ptr(p), ptr(m), ptr(v), ptr(slab), ns, n, R, C, 0.0, 0, 0, ptr(opt),
                             None, ptr(wb), ptr(wbt), s))
    t3 = timeit(lambda: call("dl_adam_dense_split3", ptr(p), ptr(m), ptr(v), ptr(slab), ns, n, R, C, 0.0, 0, 0,
                             ptr(opt), None, ptr(wb), ptr(wbt), s))
    gb = (ns + 6) * n * 4 / 1e9
    print("slabs %3d  plain %6.1f us (%5.0f GB/s)  +bf16 copies %6.1f us  +s3 planes %6.1f us" %
          (ns, t0, gb / t0 * 1e6, t1, t3), flush=True)
