"""Summarise a gpu_profile.sh run (rocprofv3 --kernel-trace --stats + separate
--pmc FETCH_SIZE / WRITE_SIZE passes) into one JSON per kernel:

  avg_us        : rocprofv3 kernel-stats average duration
  fetch_kb      : FETCH_SIZE per dispatch (KB, as rocprofv3 reports it)
  write_kb      : WRITE_SIZE per dispatch (KB)
  hbm_bytes     : (2 * FETCH_SIZE + WRITE_SIZE) * 1024 — MI355X_MICROARCH.md §HBM: on
                  gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
                  streaming read (16 B/lane); exact for the streaming Adam sweep, an
                  upper-bound-style estimate for other access widths (uncalibrated).

usage: python scripts/pmc_summary.py gpurun_out/r01e profiles/r01e/pmc_summary.json [workload] [id_dist]
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^void ", "", name)
    return name.replace("dl::", "")


def main(src, dst, workload="c2", id_dist="uniform"):
    stats = {}
    p = os.path.join(src, "prof_trace", "trace_kernel_stats.csv")
    for r in csv.DictReader(open(p)):
        stats[short(r["Name"])] = {"avg_us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"])}
    for ctr, sub in (("FETCH_SIZE", "prof_fetch/fetch_counter_collection.csv"),
                     ("WRITE_SIZE", "prof_write/write_counter_collection.csv")):
        acc = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, sub))):
            if r["Counter_Name"] == ctr:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            stats.setdefault(k, {})[ctr.lower().replace("_size", "_kb")] = sum(v) / len(v)
    for k, v in stats.items():
        if "fetch_kb" in v and "write_kb" in v:
            v["hbm_bytes"] = (2 * v["fetch_kb"] + v["write_kb"]) * 1024
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump({"source": src, "workload": workload, "id_dist": id_dist, "kernels": stats}, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1].get("avg_us", 0))[:14]:
        print("%-60s %10.1f us  hbm %s" % (k[:60], v.get("avg_us", 0), "%.3g GB" % (v["hbm_bytes"] / 1e9)
                                          if "hbm_bytes" in v else "-"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *sys.argv[3:5])
