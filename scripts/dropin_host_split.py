"""Host-side costs of one C5 load-style batch (the Wide&Deep drop-in's loop, wdl.py:296): the
unpickle, the array conversions and the pageable host-to-device copies of its 31 MB, each timed
alone (median of 10) — where the drop-in's step time above the engine's goes.

    python scripts/dropin_host_split.py
"""
import os
import pickle
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd.synthetic import make_batch  # noqa: E402

B = 65536
b = make_batch(B, cate_index_size=26_000_000, seed=500, wide_fields=26)
d = {"labels": b["label"], "cont_feats": b["cont_feats"], "cate_feats": b["cate_feats"], "wide_feats": b["wide_feats"]}
for proto in (4, 5):
    item = pickle.dumps(d, protocol=proto)
    t = []
    for _ in range(10):
        t0 = time.perf_counter()
        pickle.loads(item)
        t.append(time.perf_counter() - t0)
    print("unpickle protocol %d: %.1f MB, %.3f ms" % (proto, len(item) / 1e6, statistics.median(t) * 1e3))
u = pickle.loads(pickle.dumps(d, protocol=5))
dev = {k: torch.empty(v.shape, dtype=torch.from_numpy(np.ascontiguousarray(v)).dtype, device="cuda")
       for k, v in u.items()}
torch.cuda.synchronize()
for name, nb in (("pageable", False), ("pinned", True)):
    src = {k: (torch.from_numpy(v).pin_memory() if nb else torch.from_numpy(v)) for k, v in u.items()}
    t = []
    for _ in range(10):
        t0 = time.perf_counter()
        for k in src:
            dev[k].copy_(src[k], non_blocking=nb)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    print("host-to-device %s: %.3f ms" % (name, statistics.median(t) * 1e3))
t = []
for _ in range(10):
    t0 = time.perf_counter()
    pinned = {k: torch.empty(v.shape, dtype=dev[k].dtype).pin_memory() for k, v in u.items()} if not t else pinned
    for k, v in u.items():
        pinned[k].numpy()[...] = v
    t.append(time.perf_counter() - t0)
print("copy into pinned buffers: %.3f ms" % statistics.median(t[1:]))
