"""Library yardstick for the tower GEMMs (a MEASUREMENT only, never the product path):
torch.matmul (hipBLASLt / rocBLAS under PyTorch-ROCm) at exactly the shapes our hand-written
kernels run — C5's bf16 tower (forward, dX, dW; batch 65,536, K = 432 / 400, N = 400) and C2's
fp32 tower (the same shapes in f32; ours run them as six bf16 plane products, gemm_s3.hip) —
beside our own kernels through the C ABI (scripts/gemm_bf16_bench.py's calls).  HIP events, median
of reps.  python scripts/gemm_yardstick.py [reps] > profiles/<tag>/gemm_yardstick.json"""
import json
import sys

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = 65536
dev = "cuda"


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    v = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
    return v[len(v) // 2]


res = {}
for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "f32")):
    x0 = torch.randn(B, 432, device=dev, dtype=dt)
    h = torch.randn(B, 400, device=dev, dtype=dt)
    W0 = torch.randn(432, 400, device=dev, dtype=dt)
    W1 = torch.randn(400, 400, device=dev, dtype=dt)
    cases = {
        "fwd_l0 [B,432]x[432,400]": (lambda: torch.matmul(x0, W0), 2 * B * 432 * 400),
        "fwd_l1 [B,400]x[400,400]": (lambda: torch.matmul(h, W1), 2 * B * 400 * 400),
        "dx_l1 [B,400]x[400,400]^T": (lambda: torch.matmul(h, W1.t()), 2 * B * 400 * 400),
        "dx_l0 [B,400]x[432,400]^T": (lambda: torch.matmul(h, W0.t()), 2 * B * 400 * 432),
        "dw_l0 [432,B]x[B,400]": (lambda: torch.matmul(x0.t(), h), 2 * B * 432 * 400),
        "dw_l1 [400,B]x[B,400]": (lambda: torch.matmul(h.t(), h), 2 * B * 400 * 400),
    }
    for name, (fn, fl) in cases.items():
        us = timeit(fn)
        res["torch.matmul %s %s" % (tag, name)] = {"us": round(us, 1), "TFLOP/s": round(fl / us / 1e6, 1)}
        print("torch.matmul %-5s %-28s %8.1f us %7.1f TF/s" % (tag, name, us, fl / us / 1e6), file=sys.stderr, flush=True)
    del x0, h, W0, W1
    torch.cuda.empty_cache()

# ours: the C5 bf16 kernels (dl_gemm_bf16) at the same shapes as the engine calls them
s = _lib.stream_handle()
bf = lambda *sh: torch.randn(*sh, device=dev).to(torch.bfloat16)
x0 = bf(B, 432)
hb = bf(B, 416)
WT0 = bf(400, 432)
W1b = bf(416, 400)
WT1 = bf(400, 416)
out_b = torch.zeros(B, 416, device=dev, dtype=torch.bfloat16)
out_f = torch.zeros(B, 432, device=dev)
slab = torch.zeros(96 * 432 * 416, device=dev)
ours = {
    "ours bf16 fwd_l0 (relu, bf16 out)": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 432, ptr(x0), 432, ptr(WT0), 432,
                                                       ptr(out_b), 416, 1, 1, None, 0, 1, 0, s), 2 * B * 433 * 400),
    "ours bf16 fwd_l1 (relu, bf16 out)": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 400, ptr(hb), 416, ptr(WT1), 416,
                                                       ptr(out_b), 416, 1, 1, None, 0, 1, 0, s), 2 * B * 401 * 400),
    "ours bf16 dx_l1 (relu-grad mask, bf16 out)": (lambda: call("dl_gemm_bf16", 0, 1, B, 400, 400, ptr(hb), 416,
                                                                ptr(W1b), 400, ptr(out_b), 416, 1, 2, ptr(hb), 416, 1,
                                                                0, s), 2 * B * 400 * 400),
    "ours bf16 dx_l0 (f32 out)": (lambda: call("dl_gemm_bf16", 0, 1, B, 432, 400, ptr(hb), 416, ptr(W1b), 400,
                                               ptr(out_f), 432, 0, 0, None, 0, 1, 0, s), 2 * B * 400 * 432),
    "ours bf16 dw_l0 (split 85)": (lambda: call("dl_gemm_bf16", 1, 0, 432, 400, B, ptr(x0), 432, ptr(out_b), 416,
                                                ptr(slab), 400, 0, 3, None, 0, 85, 432 * 400, s), 2 * B * 433 * 400),
}
for name, (fn, fl) in ours.items():
    us = timeit(fn)
    res[name] = {"us": round(us, 1), "TFLOP/s": round(fl / us / 1e6, 1)}
    print("%-44s %8.1f us %7.1f TF/s" % (name, us, fl / us / 1e6), file=sys.stderr, flush=True)
print(json.dumps({"reps": reps, "batch": B, "device": torch.cuda.get_device_name(0), "median_us": res}))
