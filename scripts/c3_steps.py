"""A short C3 (deepfm_multi_cate, 6 multi-hot slots x 60) training run for counter passes: the
engine at bench.py's C3 shapes, `age` graph steps to bring row lags to steady state, then `steps`
more — the program a rocprofv3 --pmc pass wraps (FETCH_SIZE / WRITE_SIZE per kernel dispatch).
python scripts/c3_steps.py [steps] [age]   (DLAMD_VARIANT picks a diagnostics build)"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from deep_learning_amd.engine import CTREngine  # noqa: E402
from deep_learning_amd.synthetic import make_batch_device  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
age = int(sys.argv[2]) if len(sys.argv) > 2 else 24
B = bench.C2["B"]
spec = bench.make_spec("c3", bench.C2["per_field_vocab"])
eng = CTREngine(spec, max_batch=B, seed=2019, adam="lazy")
kw = dict(cont=0, cate_fields=bench.C2["S"], cate_index_size=spec.cate_index_size, multi_slots=6, multi_width=60,
          cate_only=True)
batches = [make_batch_device(B, seed=i, **kw) for i in range(4)]
for i in range(age + steps):
    eng.train_step(batches[i % 4], graph=True, next_batch=batches[(i + 1) % 4])
torch.cuda.synchronize()
print("c3 steps done, loss %.5f" % eng.loss(), flush=True)
