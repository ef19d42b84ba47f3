"""Diagnose the sharded chain update at one rank (RCCL): per-step sync and chain checks."""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd.engine import ModelSpec  # noqa: E402
from deep_learning_amd.shard import Exchange, ShardedCTREngine  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
vocab = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
spec = ModelSpec("deepfm_pipeline", C=13, V=0, S=26, E=16, cate_index_size=26 * vocab, hidden=[400, 400, 400])
eng = ShardedCTREngine(spec, B, Exchange(), seed=1, adam="lazy")
eng.init_device(1)
bs = [{k: torch.from_numpy(v).cuda() for k, v in make_batch(B, cate_index_size=spec.cate_index_size, seed=i).items()}
      for i in range(3)]
for step in range(6):
    t0 = time.time()
    eng.train_step(bs[step % 3], graph=step >= 2)
    print("step", step, "launched", flush=True)
    torch.cuda.synchronize()
    h = eng.own_head
    print("step %d done %.3fs; heads != -1: %d; loss %.5f" % (step, time.time() - t0, int((h != -1).sum()),
                                                               eng.loss()), flush=True)
dist.destroy_process_group()
