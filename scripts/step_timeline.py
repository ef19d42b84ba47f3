"""Training-step timelines from a rocprofv3 --kernel-trace CSV of bench.py.

    python scripts/step_timeline.py trace.csv [step]

Steps are delimited by dl::step_begin_kernel launches.  Prints, for every step: its duration,
the time the compute queue was busy, the kernels on other queues (the prefetched index build)
and the summed gaps between the compute queue's kernels; then the kernel-by-kernel timeline of
one step (default: the median-duration step of the first half — the hipGraph replays of the
timed region come before bench.py's eager per-kernel steps)."""
import csv
import statistics
import sys


def main(path, pick=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "step_begin" in r["Kernel_Name"]]
    if len(starts) < 2:
        print("fewer than two steps in the trace")
        return
    main_q = rows[starts[0]]["Queue_Id"]
    steps = []
    for a, b in zip(starts[:-1], starts[1:]):
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy, gaps, side, prev = 0, 0, 0, t0
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if r["Queue_Id"] != main_q:
                side += e - s
                continue
            if s > prev:
                gaps += s - prev
            busy += max(0, min(e, t1) - max(s, prev))
            prev = max(prev, e)
        steps.append((a, b, (t1 - t0) / 1e3, busy / 1e3, gaps / 1e3, side / 1e3))
    for k, (a, b, dur, busy, gaps, side) in enumerate(steps):
        print("step %3d: %8.1f us, compute queue busy %8.1f, gaps %6.1f, other queues %7.1f us of kernels"
              % (k, dur, busy, gaps, side))
    if pick is None:
        half = steps[: max(1, len(steps) // 2)]
        med = statistics.median(s[2] for s in half)
        pick = min(range(len(half)), key=lambda k: abs(half[k][2] - med))
    a, b = steps[pick][0], steps[pick][1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev = {}
    print("\nstep %d" % pick)
    for r in rows[a:b]:
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
        print("%8.1f gap %7.1f dur %7.1f  q%s %s" % ((s - t0) / 1e3, (s - prev.get(q, t0)) / 1e3, (e - s) / 1e3, q,
                                                     r["Kernel_Name"][:90]))
        prev[q] = max(prev.get(q, t0), e)


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
