"""Finds the first step where the lazy (row-record) engine and the dense-sorted
engine diverge, and which parameters/rows differ (GPU diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from deep_learning_amd.engine import CTREngine, ModelSpec
from tests.test_gpu_parity import CASES, _batches, _model

name = sys.argv[1] if len(sys.argv) > 1 else "deepfm_pipeline"
hist = int(sys.argv[2]) if len(sys.argv) > 2 else 8
kw = dict(CASES[name], cate_index_size=50000)
spec = ModelSpec(_model(name), **kw)
dense = CTREngine(spec, max_batch=128, seed=3, bwd="sorted")
lazy = CTREngine(spec, max_batch=128, seed=3, adam="lazy", hist_len=hist)
bs = _batches(name, kw, 128, 21, seed=7)
tabk = "weight_mat" if spec.model == "wdl" else "feats_emb"
for i, b in enumerate(bs):
    dense.train_step(b, graph=False)
    lazy.train_step(b, graph=False)
    torch.cuda.synchronize()
    zd, zl = dense.z[:128].cpu().numpy(), lazy.z[:128].cpu().numpy()
    pd, pl = dense.params(), lazy.params()
    sd, sl = dense.adam_state(), lazy.adam_state()
    bad = [k for k in pd if not np.array_equal(pd[k], pl[k])] + \
          ["adam_" + k for k in sd if not np.array_equal(sd[k], sl[k])]
    print("step %d: logits diff %d, since_flush %d, differing: %s" %
          (i, int((zd != zl).sum()), lazy.since_flush, bad))
    if bad:
        ids = np.asarray(b["cate_feats"])
        ref_rows = set((ids + spec.C).ravel().tolist()) | set(ids.ravel().tolist())
        for k in bad:
            a, c = (pd[k], pl[k]) if k in pd else (sd[k[5:]], sl[k[5:]])
            a2, c2 = a.reshape(a.shape[0], -1), c.reshape(c.shape[0], -1)
            rows = np.nonzero((a2 != c2).any(1))[0]
            print("  %s: %d rows differ, first %s; in batch: %s; max |d| %.3g" %
                  (k, len(rows), rows[:8].tolist(), [int(r) in ref_rows for r in rows[:8]],
                   float(np.abs(a2 - c2).max())))
        break
