"""Print one training step's kernel timeline (gaps, durations) from a rocprofv3
--kernel-trace CSV.  Usage: python scripts/step_timeline.py trace.csv [step_from_end]"""
import csv
import sys


def main(path, back=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_begin" in r["Kernel_Name"]]
    i0, i1 = idx[-back - 1], idx[-back]
    t0 = int(rows[i0]["Start_Timestamp"])
    prev = t0
    busy = 0.0
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%8.1f gap %7.1f dur %7.1f  q%s %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, r["Queue_Id"],
                                                     r["Kernel_Name"][:80]))
        busy += (min(e, int(rows[i1]["Start_Timestamp"])) - max(s, prev)) / 1e3 if e > prev else 0
        prev = max(prev, e)
    print("step %.1f us, busy %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, busy))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
