"""The three-plane split GEMMs (gemm_s3.hip) against fp64 and against the f32 kernels, at
the C2 tower's shapes: relative error and time (HIP events).  python scripts/s3_bench.py [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
only = sys.argv[2] if len(sys.argv) > 2 else None   # run one case (profiling); "t:<case>": time just it
timed = None
if only and only.startswith("t:"):
    timed, only = only[2:], None
B = 65536
s = _lib.stream_handle()
g = torch.Generator(device="cuda").manual_seed(0)
z = lambda *sh: torch.randn(*sh, device="cuda", generator=g)
x0 = z(B, 432)
h = torch.relu(z(B, 416))
dy = z(B, 416) * 1e-3
W0 = z(432, 400) * 0.05
W1 = z(416, 400) * 0.05
u16 = lambda n: torch.zeros(n, dtype=torch.int16, device="cuda")
# planes: forward B = W^T [400][K] ; dX B = W [K][400]
W0T_p = u16(3 * 400 * 432)
W1T_p = u16(3 * 400 * 416)
W1_p = u16(3 * 416 * 400)
call("dl_split3", ptr(W0), 432, 400, 400, 1, ptr(W0T_p), 432, 400 * 432, s)
call("dl_split3", ptr(W1), 416, 400, 400, 1, ptr(W1T_p), 416, 400 * 416, s)
call("dl_split3", ptr(W1), 416, 400, 400, 0, ptr(W1_p), 400, 416 * 400, s)
out = torch.zeros(B, 416, device="cuda")
out2 = torch.zeros(B, 416, device="cuda")
slab = torch.zeros(160 * 432 * 400, device="cuda")   # room for every split count swept below (<= 128 slabs)


def rel(a, ref):
    return float(((a.double() - ref).abs().max() / ref.abs().max()).item())


def timeit(fn):
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


cases = []
# forward l0: h = relu(x0 . W0)
ref = torch.relu(x0.double() @ W0.double())
cases.append(("fwd_l0", 2 * B * 432 * 400,
              lambda: call("dl_gemm_s3_nt", B, 400, 432, ptr(x0), 432, ptr(W0T_p), 432, 400 * 432, ptr(out), 416, 1,
                           None, 0, s),
              lambda: call("dl_gemm_f32", 0, 0, B, 400, 432, ptr(x0), 432, ptr(W0), 400, ptr(out2), 416, 1, None, 0,
                           1, 0, s),
              lambda: (rel(out[:, :400], ref), rel(out2[:, :400], ref))))
ref1 = torch.relu(h[:, :416].double() @ W1.double())
cases.append(("fwd_l1", 2 * B * 416 * 400,
              lambda: call("dl_gemm_s3_nt", B, 400, 416, ptr(h), 416, ptr(W1T_p), 416, 400 * 416, ptr(out), 416, 1,
                           None, 0, s),
              lambda: call("dl_gemm_f32", 0, 0, B, 400, 416, ptr(h), 416, ptr(W1), 400, ptr(out2), 416, 1, None, 0,
                           1, 0, s),
              lambda: (rel(out[:, :400], ref1), rel(out2[:, :400], ref1))))
# dX l1: dx = (dy . W1^T) * (h > 0)   (K = 400 output columns of the layer, N = 416 inputs)
W1T = W1.t().contiguous()
refd = (dy[:, :400].double() @ W1.double().t()) * (h > 0).double()
cases.append(("dx_l1", 2 * B * 400 * 416,
              lambda: call("dl_gemm_s3_nt", B, 416, 400, ptr(dy), 416, ptr(W1_p), 400, 416 * 400, ptr(out), 416, 2,
                           ptr(h), 416, s),
              lambda: call("dl_gemm_f32", 0, 0, B, 416, 400, ptr(dy), 416, ptr(W1T), 416, ptr(out2), 416, 2, ptr(h),
                           416, 1, 0, s),
              lambda: (rel(out, refd), rel(out2, refd))))
# dX l1 with the ReluGrad mask from the forward's sign bitmask (dl_gemm_s3_nt_bits, epi 3)
hbits = torch.zeros(B, 32, dtype=torch.int16, device="cuda")
call("dl_gemm_s3_nt_bits", B, 400, 416, ptr(h), 416, ptr(W1T_p), 416, 400 * 416, ptr(out2), 416, 1, None, 0,
     ptr(hbits), 32, s)   # any ReLU output will do as the bitmask source for timing
cases.append(("dx_l1 bits", 2 * B * 400 * 416,
              lambda: call("dl_gemm_s3_nt_bits", B, 416, 400, ptr(dy), 416, ptr(W1_p), 400, 416 * 400, ptr(out), 416,
                           3, None, 0, ptr(hbits), 32, s),
              lambda: None,
              lambda: (0.0, 0.0)))
# dW l0: slabs of x0^T . dy
refw = x0.double().t() @ dy[:, :400].double()
slab2 = torch.zeros(64 * 432 * 400, device="cuda")
cases.append(("dw_l0", 2 * B * 432 * 400,
              lambda: call("dl_gemm_s3_tn", 432, 400, B, ptr(x0), 432, ptr(dy), 416, ptr(slab), 400, 64, 432 * 400, s),
              lambda: call("dl_gemm_f32", 1, 0, 432, 400, B, ptr(x0), 432, ptr(dy), 416, ptr(slab2), 400, 3, None, 0,
                           64, 432 * 400, s),
              lambda: (rel(slab[:64 * 432 * 400].view(64, 432, 400).sum(0), refw), rel(slab2[:64 * 432 * 400].view(64, 432, 400).sum(0), refw))))
refw1 = h.double().t() @ dy[:, :400].double()
cases.append(("dw_l1", 2 * B * 416 * 400,
              lambda: call("dl_gemm_s3_tn", 416, 400, B, ptr(h), 416, ptr(dy), 416, ptr(slab), 400, 64, 416 * 400, s),
              lambda: call("dl_gemm_f32", 1, 0, 416, 400, B, ptr(h), 416, ptr(dy), 416, ptr(slab2), 400, 3, None, 0,
                           64, 416 * 400, s),
              lambda: (rel(slab[:64 * 416 * 400].view(64, 416, 400).sum(0), refw1),
                       rel(slab2[:64 * 416 * 400].view(64, 416, 400).sum(0), refw1))))
for name, fl, f_s3, f_f32, err in cases:
    if only:
        if name == only:
            for _ in range(reps):
                f_s3()
            torch.cuda.synchronize()
            print(name, "done")
        continue
    if timed and name != timed:
        continue
    f_s3()
    f_f32()
    torch.cuda.synchronize()
    e_s3, e_f32 = err()
    t_s3, t_f32 = timeit(f_s3), (timeit(f_f32) if not timed else 1.0)
    print("%-7s s3 %7.1f us %6.1f TF/s err %.2e | f32 %7.1f us %6.1f TF/s err %.2e" %
          (name, t_s3, fl / t_s3 / 1e6, e_s3, t_f32, fl / t_f32 / 1e6, e_f32), flush=True)
for sp in (() if (only or timed) else (32, 48, 64, 96, 128)):
    fn = lambda: call("dl_gemm_s3_tn", 416, 400, B, ptr(h), 416, ptr(dy), 416, ptr(slab), 400, sp, 416 * 400, s)
    t = timeit(fn)
    print("dw_l1 s3 splits %3d %7.1f us %6.1f TF/s" % (sp, t, 2 * B * 416 * 400 / t / 1e6), flush=True)
