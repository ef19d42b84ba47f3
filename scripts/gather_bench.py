"""Record-gather microbenchmark (C2 or C5 shape): the gather is read-only on the records, so
one batch's gather is timed repeatedly at the table's natural lag after `age` training steps
over 32 distinct batches, then again right after a full flush (no catch-up at all).

    DLAMD_VARIANT=<v> python scripts/gather_bench.py [c2|c5] [age]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd.engine import C_ref, CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
age = int(sys.argv[2]) if len(sys.argv) > 2 else 64
B = 65536
if wl == "c2":
    spec = ModelSpec("deepfm_pipeline", C=13, V=0, S=26, E=16, cate_index_size=26_000_000, hidden=[400, 400, 400])
    vocab = 26_000_000
else:
    spec = ModelSpec("wdl", C=13, V=0, S=26, E=16, cate_index_size=26_000_000, hidden=[400, 400, 400], Fw=26,
                     tower="bf16")
    vocab = 26_000_000
eng = CTREngine(spec, max_batch=B, seed=2019, adam="lazy")
bs = []
for i in range(32):
    b = make_batch(B, cate_index_size=vocab, seed=100 + i, wide_fields=spec.Fw)
    bs.append({k: torch.from_numpy(v).cuda() for k, v in b.items()})
for i in range(age):
    eng.train_step(bs[i % 32], graph=False)
torch.cuda.synchronize()


def time_gather(label, reps=10):
    eng._begin(bs[age % 32])
    eng._pre(B)
    s = _lib.stream_handle()
    L = eng.layout
    L.batch = B
    args = (C_ref(L), ptr(eng.rec), eng.rec_ld, eng.rec_flags, eng.n_rep, ptr(eng.idx_uniq), ptr(eng.idx_n),
            B * eng.n_slot, 1, ptr(eng.hist), eng.hist_len, ptr(eng.opt), 0, ptr(eng.rows_u), ptr(eng.rows_u1),
            ptr(eng.mv_u), s)
    call("dl_rec_gather", *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call("dl_rec_gather", *args)
    e1.record()
    torch.cuda.synchronize()
    nu = int(eng.idx_n[0].item())
    print("%-6s %-14s U=%d  %.1f us" % (os.environ.get("DLAMD_VARIANT", "cur"), label, nu,
                                        e0.elapsed_time(e1) * 1e3 / reps), flush=True)
    return eng.rows_u[: eng.n_rep + nu].clone(), eng.mv_u[: eng.n_rep + nu].clone()


r1, m1 = time_gather("natural lag")
eng.flush()
r2, m2 = time_gather("after flush")
print("caught-up rows equal:", bool(torch.equal(r1, r2)), bool(torch.equal(m1, m2)), flush=True)
