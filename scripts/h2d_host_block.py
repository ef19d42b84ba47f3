"""Does an asynchronous host-to-device copy from pinned memory return before the DMA ends?
Host time of dst.copy_(pinned, non_blocking=True) for the C5 drop-in's fields (31 MB a batch),
on the current and on a side stream, against the copies' device time.
    python scripts/h2d_host_block.py"""
import statistics
import time

import torch

sizes = {"label": (65536, 4), "cont": (65536 * 13, 4), "cate": (65536 * 26, 8), "wide": (65536 * 26, 8)}
src = {k: torch.empty(n, dtype=torch.float32 if b == 4 else torch.int64).pin_memory() for k, (n, b) in sizes.items()}
dst = {k: torch.empty_like(v, device="cuda") for k, v in src.items()}
side = torch.cuda.Stream()
for name, st in (("current stream", torch.cuda.current_stream()), ("side stream", side)):
    host, wall = [], []
    for i in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            for k in src:
                dst[k].copy_(src[k], non_blocking=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i >= 5:
            host.append(t1 - t0)
            wall.append(t2 - t0)
    print("%-15s host return %.3f ms, copies done %.3f ms" % (name, statistics.median(host) * 1e3,
                                                              statistics.median(wall) * 1e3))
# behind a busy stream: the copies queued after 2 ms of device work
a = torch.randn(4096, 4096, device="cuda")
host = []
for i in range(15):
    torch.cuda.synchronize()
    for _ in range(4):
        a = a @ a / 64.0
    t0 = time.perf_counter()
    for k in src:
        dst[k].copy_(src[k], non_blocking=True)
    host.append(time.perf_counter() - t0)
print("behind queued work: host return %.3f ms" % (statistics.median(host[5:]) * 1e3))
# a side stream that waits on an event of the busy stream, then copies (the engine's prefetch)
host, wait_host = [], []
for i in range(15):
    torch.cuda.synchronize()
    for _ in range(4):
        a = a @ a / 64.0
    ev = torch.cuda.Event()
    ev.record()
    t0 = time.perf_counter()
    side.wait_event(ev)
    t1 = time.perf_counter()
    with torch.cuda.stream(side):
        for k in src:
            dst[k].copy_(src[k], non_blocking=True)
    host.append(time.perf_counter() - t1)
    wait_host.append(t1 - t0)
print("side stream behind a cross-stream event: wait_event %.3f ms, copies' host return %.3f ms"
      % (statistics.median(wait_host[5:]) * 1e3, statistics.median(host[5:]) * 1e3))
# the matmuls alone, for scale
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(4):
    a = a @ a / 64.0
torch.cuda.synchronize()
print("the 4 queued products take %.3f ms on the device" % ((time.perf_counter() - t0) * 1e3))
# the first copy after the copy path has been idle (the drop-in's epoch start)
for idle in (0.002, 0.01, 0.05, 0.2):
    r = []
    for i in range(6):
        torch.cuda.synchronize()
        time.sleep(idle)
        t0 = time.perf_counter()
        with torch.cuda.stream(side):
            dst["label"].copy_(src["label"], non_blocking=True)
        r.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    print("after %.0f ms idle: first copy's host return %s ms" % (idle * 1e3, [round(x * 1e3, 3) for x in r]))
# the side stream behind an event that follows host-to-device copies on the current stream (the
# drop-in's first step of an epoch: its batch staged on the compute stream, the next one prefetched)
r = []
big = {k: v for k, v in src.items() if k != "label"}
for i in range(8):
    torch.cuda.synchronize()
    for k in big:
        dst[k].copy_(big[k], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    side.wait_event(ev)
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        dst["label"].copy_(src["label"], non_blocking=True)
    r.append(time.perf_counter() - t0)
print("side copy behind the current stream's copies: host return %s ms" % [round(x * 1e3, 3) for x in r])
r = []
for i in range(8):
    torch.cuda.synchronize()
    for k in big:
        dst[k].copy_(big[k], non_blocking=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        dst["label"].copy_(src["label"], non_blocking=True)
    r.append(time.perf_counter() - t0)
print("side copy beside (no dependency on) the current stream's copies: host return %s ms" % [round(x * 1e3, 3) for x in r])
