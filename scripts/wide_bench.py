"""Wide-record gather microbenchmark (C5 shape): dl_wide_rec_gather is read-only on the wide
records, so one batch's gather is timed repeatedly at the table's natural lag after `age`
training steps, then again right after a full flush (no replay at all) — the replay's cost.

    DLAMD_VARIANT=<v> python scripts/wide_bench.py [age]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

age = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = 65536
vocab = 26_000_000
spec = ModelSpec("wdl", C=13, V=0, S=26, E=16, cate_index_size=vocab, hidden=[400, 400, 400], Fw=26, tower="bf16")
eng = CTREngine(spec, max_batch=B, seed=2019, adam="lazy")
bs = []
for i in range(32):
    b = make_batch(B, cate_index_size=vocab, seed=100 + i, wide_fields=spec.Fw)
    bs.append({k: torch.from_numpy(v).cuda() for k, v in b.items()})
for i in range(age):
    eng.train_step(bs[i % 32], graph=False)
torch.cuda.synchronize()


def time_gather(label, reps=20):
    eng._begin(bs[age % 32])
    eng._pre(B)
    s = _lib.stream_handle()
    H = spec.hidden[-1]
    nw = B * spec.Fw
    args = (ptr(eng.wrec), eng.w_rows, ptr(eng.widx_uniq), ptr(eng.widx_n), nw, spec.Fw, H, ptr(eng.hist),
            eng.hist_len, ptr(eng.opt), spec.l2, 1, ptr(eng.wloc), ptr(eng.wstash), ptr(eng.wrep), s)
    call("dl_wide_rec_gather", *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call("dl_wide_rec_gather", *args)
    e1.record()
    torch.cuda.synchronize()
    nu = int(eng.widx_n[0].item())
    print("%-6s %-14s U=%d  %.1f us" % (os.environ.get("DLAMD_VARIANT", "cur"), label, nu,
                                        e0.elapsed_time(e1) * 1e3 / reps), flush=True)
    return eng.wstash[:nu].clone(), eng.wloc[: spec.Fw + H + nu].clone()


s1, w1 = time_gather("natural lag")
eng.flush()
s2, w2 = time_gather("after flush")
print("caught-up rows equal:", bool(torch.equal(s1, s2)), bool(torch.equal(w1, w2)), flush=True)
