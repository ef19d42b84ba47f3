"""Where the drop-in loop's host time goes with the native-decoded feed (DLAMD_PINNED_FEED=1):
the main thread's wait for the next decoded batch, its train_step call (staging + launches), and
the decode time on the worker threads.  python scripts/dropin_feed_timing.py [n_batches]"""
import os
import sys
import time
import types

import torch

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
    if T["n"] == 0:   # host: epoch start -> the first step's call, and that call's own time
        T["first_in"], T["first_call"] = t0 - T["t_epoch"], time.perf_counter() - t0
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
FIRST = {}   # per engine method: host ms inside the epoch's first train_step call
LATER = {}   # and summed over the later calls


def _wrap(name):
    f = getattr(CTREngine, name)

    def g(self, *a, **k):
        t0 = time.perf_counter()
        r = f(self, *a, **k)
        dt = (time.perf_counter() - t0) * 1e3
        if T["n"] == 0:
            FIRST[name] = FIRST.get(name, 0.0) + dt
        else:
            LATER[name] = LATER.get(name, 0.0) + dt
        return r
    setattr(CTREngine, name, g)


import deep_learning_amd.engine as _engmod  # noqa: E402
_ci = _engmod._copy_in


def _timed_copy_in(dst, x, dtype, dev):
    t0 = time.perf_counter()
    pinned = isinstance(x, torch.Tensor) and x.is_pinned()
    t1 = time.perf_counter()
    _ci(dst, x, dtype, dev)
    if T["n"] == 0:
        FIRST.setdefault("copy_in", []).append(round((time.perf_counter() - t0) * 1e3, 3))
        FIRST.setdefault("is_pinned", []).append((pinned, round((t1 - t0) * 1e3, 3)))


_engmod._copy_in = _timed_copy_in
for _m in ("_begin", "prefetch", "_capture", "_release", "_queue_status", "flush", "stage"):
    if hasattr(CTREngine, _m):
        _wrap(_m)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
_epoch = ls.LoadStyleModel.train_epoch
passes = []


def timed_epoch(self, items):
    for k in list(T):
        T[k] = 0 if k == "n" else 0.0
    FIRST.clear()
    LATER.clear()
    eng = self.model_optimizer()
    eng.step_events = []          # the compute stream's step spans and the gaps between steps
    import torch
    e_begin = torch.cuda.Event(enable_timing=True)
    e_end = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    T["t_epoch"] = t0
    e_begin.record()
    r = _epoch(self, items)
    e_end.record()
    torch.cuda.synchronize()
    ev, eng.step_events = eng.step_events, None
    starts = [e for k, e in ev if k == 0]
    ends = [e for k, e in ev if k == 1]
    span = [a.elapsed_time(b) for a, b in zip(starts, ends)]
    gap = [b.elapsed_time(a) for b, a in zip(ends, starts[1:])]
    T["span"] = sum(span) / max(1, len(span))
    T["gap"] = sum(gap) / max(1, len(gap))
    T["lead"] = e_begin.elapsed_time(starts[0]) if starts else 0.0    # feed startup: first batch decoded
    T["tail"] = ends[-1].elapsed_time(e_end) if ends else 0.0
    T["steps_ev"] = len(span)
    passes.append((time.perf_counter() - t0, dict(T)))
    return r


ls.LoadStyleModel.train_epoch = timed_epoch
r = bench.dropin_fit(types.SimpleNamespace(batch=65536), n_batches=n)
dt, t = passes[-1]
steps = t["n"]
print("ms/step %.3f (pass %.3f) | per step: wait %.3f, train_step %.3f (ring wait %.3f), decode (workers) %.3f ms"
      % (r["ms_per_step"], dt / steps * 1e3, t["wait"] / steps * 1e3, t["step"] / steps * 1e3, t["ring"] / steps * 1e3,
         t["decode"] / steps * 1e3))
print("compute stream: step span %.3f ms, gap to the next step %.3f ms over %d steps; before the first step "
      "%.3f ms, after the last %.3f ms" % (t["span"], t["gap"], t["steps_ev"], t["lead"], t["tail"]))
print("host: epoch start -> first train_step %.3f ms, its call %.3f ms" % (t["first_in"] * 1e3, t["first_call"] * 1e3))
print("host: inside the first train_step (ms):", {k: (round(v, 3) if not isinstance(v, list) else v) for k, v in FIRST.items()})
print("host: per later train_step (ms):", {k: round(v / max(1, steps - 1), 3) for k, v in LATER.items()})
