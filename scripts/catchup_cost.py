"""How much of the record kernels' time is the lazy catch-up: C2, per-kernel HIP-event
times for a step at the natural lag (~20 steps in) and for a step right after a full
flush (every row's lag = 1).  python scripts/catchup_cost.py [fwd_rec 0|1]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402

fwd_rec = bool(int(sys.argv[1])) if len(sys.argv) > 1 else False
B = 65536
spec = ModelSpec("deepfm_pipeline", C=13, V=0, S=26, E=16, cate_index_size=26_000_000, hidden=[400, 400, 400])
eng = CTREngine(spec, max_batch=B, seed=2019, adam="lazy", fwd_rec=fwd_rec)
bs = [{k: torch.from_numpy(v).cuda() for k, v in make_batch(B, cate_index_size=26_000_000, seed=i).items()}
      for i in range(4)]


def timed(i, label):
    eng.prof = []
    eng.train_step(bs[i % 4], graph=False)
    torch.cuda.synchronize()
    t = {}
    for lab, e0, e1 in eng.prof:
        t[lab] = t.get(lab, 0.0) + e0.elapsed_time(e1) * 1e3
    eng.prof = None
    print(label, {k: round(v, 1) for k, v in t.items() if k in ("rec_gather", "embed_fwd", "embed_bwd", "index_build",
                                                               "rec_flush")}, flush=True)


for i in range(20):
    eng.train_step(bs[i % 4], graph=False)
torch.cuda.synchronize()
timed(20, "natural lag  ")
timed(21, "natural lag  ")
eng.flush()
timed(22, "after flush  ")
eng.flush()
timed(23, "after flush  ")
