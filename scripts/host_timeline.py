"""Host submission against GPU execution at the step boundary, from one rocprofv3 run with
--kernel-trace --hip-runtime-trace (CSV) of bench.py.

    python scripts/host_timeline.py kernel_trace.csv hip_api_trace.csv [step]

For every step (delimited by dl::step_begin_kernel): how long before its first kernel ran the
host had submitted it (the launching API call, joined on Correlation_Id), and the host's API
time in the step.  Then, for one step (default: the median of the first half), every API call
and kernel from the previous step's last compute-queue kernel to the step's first, in time order
— a step whose first kernel starts right after its submit call is host-bound at the boundary."""
import csv
import statistics
import sys


def main(kpath, apath, pick=None):
    ks = sorted(csv.DictReader(open(kpath)), key=lambda r: int(r["Start_Timestamp"]))
    api = sorted(csv.DictReader(open(apath)), key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    starts = [i for i, r in enumerate(ks) if "step_begin" in r["Kernel_Name"]]
    if len(starts) < 3:
        print("fewer than three steps in the trace")
        return
    main_q = ks[starts[0]]["Queue_Id"]
    rows = []
    for n, (a, b) in enumerate(zip(starts[:-1], starts[1:])):
        t0, t1 = int(ks[a]["Start_Timestamp"]), int(ks[b]["Start_Timestamp"])
        call = by_corr.get(ks[a]["Correlation_Id"])
        lead = (t0 - int(call["Start_Timestamp"])) / 1e3 if call else float("nan")
        prev_end = max((int(r["End_Timestamp"]) for r in ks[:a] if r["Queue_Id"] == main_q), default=t0)
        idle = (t0 - prev_end) / 1e3
        host = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in api
                   if t0 <= int(r["Start_Timestamp"]) < t1) / 1e3
        rows.append((a, b, (t1 - t0) / 1e3, idle, lead, call["Function"] if call else "?", host))
        print("step %3d: %8.1f us, idle before its first kernel %6.1f, submitted %8.1f us ahead by %s, "
              "host API time %7.1f us" % (n, (t1 - t0) / 1e3, idle, lead, rows[-1][5], host))
    if pick is None:
        half = rows[: max(1, len(rows) // 2)]
        med = statistics.median(r[2] for r in half)
        pick = min(range(1, len(half)), key=lambda k: abs(half[k][2] - med)) if len(half) > 1 else 0
    a = rows[pick][0]
    t0 = int(ks[a]["Start_Timestamp"])
    w0 = max((int(r["End_Timestamp"]) for r in ks[:a] if r["Queue_Id"] == main_q), default=t0) - 400_000
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API t%s %s" % (r["Thread_Id"], r["Function"]))
          for r in api if w0 <= int(r["Start_Timestamp"]) <= t0 + 50_000]
    for r in ks:
        s = int(r["Start_Timestamp"])
        if w0 <= s <= t0 + 50_000:
            c = by_corr.get(r["Correlation_Id"])
            via = " <- %s@%.1f" % (c["Function"], (int(c["Start_Timestamp"]) - t0) / 1e3) if c else ""
            ev.append((s, int(r["End_Timestamp"]), "K q%s %s%s" % (r["Queue_Id"], r["Kernel_Name"][:70], via)))
    ev.sort()
    print("\nstep %d boundary (us relative to its first kernel)" % pick)
    for s, e, what in ev:
        print("%9.1f dur %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, what))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
