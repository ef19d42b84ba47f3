"""Gaps between consecutive kernels on the compute stream in a rocprofv3 kernel trace: per
kernel name, its mean duration and the mean idle time before it starts (the previous kernel on
the same queue ended -> this one started), over the last N steps of the trace.
    python scripts/trace_gaps.py <kernel_trace.csv> [first_kernel_of_step]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "step_begin"
by_q = defaultdict(list)
for r in rows:
    q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
    by_q[q].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
q, ks = max(by_q.items(), key=lambda kv: len(kv[1]))
ks.sort()
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
steps = [i for i, k in enumerate(ks) if first in k[2]]
if len(steps) > 3:
    ks = ks[steps[-4]:steps[-1]]          # the last three whole steps
prev_end = None
for s, e, n in ks:
    name = n.split("(")[0].split("<")[0].split("::")[-1][:40]
    dur[name] += (e - s) / 1e3
    if prev_end is not None:
        gap[name] += max(0, s - prev_end) / 1e3
    cnt[name] += 1
    prev_end = e
tot_d = sum(dur.values()); tot_g = sum(gap.values())
print("queue %s: %d kernels, busy %.1f us, idle between kernels %.1f us" % (q, len(ks), tot_d, tot_g))
for name in sorted(dur, key=lambda n: -gap[n]):
    print("%-40s n=%3d  dur %8.1f us  gap-before %6.1f us" % (name, cnt[name], dur[name] / cnt[name], gap[name] / cnt[name]))
