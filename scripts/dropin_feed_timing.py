"""Where the drop-in loop's host time goes with the native-decoded feed (DLAMD_PINNED_FEED=1):
the main thread's wait for the next decoded batch, its train_step call (staging + launches), and
the decode time on the worker threads.  python scripts/dropin_feed_timing.py [n_batches]"""
import os
import sys
import time
import types

os.environ["DLAMD_PINNED_FEED"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from deep_learning_amd.models import _load_style as ls  # noqa: E402
from deep_learning_amd.engine import CTREngine  # noqa: E402

T = {"wait": 0.0, "step": 0.0, "decode": 0.0, "ring": 0.0, "n": 0}
if os.environ.get("DLAMD_SWITCH"):   # the interpreter's GIL switch interval (s), for A/B
    sys.setswitchinterval(float(os.environ["DLAMD_SWITCH"]))


class TimedFeed(ls.PinnedFeed):
    def _native(self, s, item):
        t0 = time.perf_counter()
        r = super()._native(s, item)
        T["decode"] += time.perf_counter() - t0
        return r

    def __iter__(self):
        while self.pending:
            fut = self.pending.pop(0)
            t0 = time.perf_counter()
            b = fut.result()
            T["wait"] += time.perf_counter() - t0
            self._submit()
            yield b


ls.PinnedFeed = TimedFeed
_ts = CTREngine.train_step


def timed_step(self, *a, **k):
    t0 = time.perf_counter()
    r = _ts(self, *a, **k)
    T["step"] += time.perf_counter() - t0
    T["n"] += 1
    return r


CTREngine.train_step = timed_step
_rs = CTREngine._ring_status


def timed_ring(self, *a, **k):
    t0 = time.perf_counter()
    r = _rs(self, *a, **k)
    T["ring"] += time.perf_counter() - t0
    return r


CTREngine._ring_status = timed_ring
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
_epoch = ls.LoadStyleModel.train_epoch
passes = []


def timed_epoch(self, items):
    for k in T:
        T[k] = 0 if k == "n" else 0.0
    t0 = time.perf_counter()
    r = _epoch(self, items)
    import torch
    torch.cuda.synchronize()
    passes.append((time.perf_counter() - t0, dict(T)))
    return r


ls.LoadStyleModel.train_epoch = timed_epoch
r = bench.dropin_fit(types.SimpleNamespace(batch=65536), n_batches=n)
dt, t = passes[-1]
steps = t["n"]
print("ms/step %.3f (pass %.3f) | per step: wait %.3f, train_step %.3f (ring wait %.3f), decode (workers) %.3f ms"
      % (r["ms_per_step"], dt / steps * 1e3, t["wait"] / steps * 1e3, t["step"] / steps * 1e3, t["ring"] / steps * 1e3,
         t["decode"] / steps * 1e3))
