"""Times the batch index build (dl_validate_batch + dl_index_build, CTREngine._pre) alone at a
BASELINE shape: python scripts/index_bench.py [c2|c3] [reps] — C2: B = 65,536, 52 references a
sample over 26 M rows; C3: 26 single + 6 multi-hot slots x 60 (mean 30 ids) a sample, FM + deep.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import sys
import time

import torch

sys.path.insert(0, ".")
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch_device  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B, N = 65536, 26_000_000
if wl == "c3":
    ranges = [[60 * i, 60 * (i + 1), "slot%d" % i] for i in range(6)]
    spec = ModelSpec("deepfm_multi_cate", C=0, V=0, S=26, E=16, cate_index_size=N, hidden=[16], multi_ranges=ranges)
    kw = dict(cont=0, cate_fields=26, cate_index_size=N, multi_slots=6, multi_width=60, cate_only=True)
else:
    spec = ModelSpec("deepfm_pipeline", C=13, S=26, E=16, cate_index_size=N, hidden=[16])
    kw = dict(cate_index_size=N)
eng = CTREngine(spec, max_batch=B, adam="lazy", init="none")
eng.stage(make_batch_device(B, seed=1, **kw))
for _ in range(3):
    eng._pre(B)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    eng._pre(B)
torch.cuda.synchronize()
print("%s index_build %.1f us (unique rows %d)" % (wl, (time.perf_counter() - t0) / reps * 1e6, int(eng.idx_n[0].item())))
