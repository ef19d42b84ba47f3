"""Times dl_index_build at C2 shape (B=65536, 52 refs/sample, 26M rows) — for rocprofv3 traces."""
import sys
import time

import torch

sys.path.insert(0, ".")
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402

spec = ModelSpec("deepfm_pipeline", C=13, S=26, E=16, cate_index_size=26_000_000, hidden=[16])
eng = CTREngine(spec, max_batch=65536, adam="lazy", init="none")
eng.stage(make_batch(65536, cate_index_size=26_000_000, seed=1))
for _ in range(3):
    eng._pre(65536)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    eng._pre(65536)
torch.cuda.synchronize()
print("index_build %.1f us" % ((time.perf_counter() - t0) / 20 * 1e6))
