"""SQ counter passes of scripts/pmc_s3.sh -> one JSON: per case, the s3 GEMM kernel's counters
(mean over its dispatches).  python scripts/sq_summary.py <s3pmc dir> <out.json> case...
(SQ_KERNEL=<substring> in the environment picks another kernel than gemm_s3)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, out, cases = sys.argv[1], sys.argv[2], sys.argv[3:]
want = os.environ.get("SQ_KERNEL", "gemm_s3")
res = {}
for case in cases:
    acc, kern = defaultdict(list), None
    for f in sorted(glob.glob(os.path.join(d, case + "_pass*_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if want not in row["Kernel_Name"]:
                continue
            kern = row["Kernel_Name"]
            acc[(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), vals in acc.items():
        per[name].append(sum(vals))
    res[case] = {"kernel": kern, "counters": {k: sum(v) / len(v) for k, v in per.items()},
                 "dispatches": max((len(v) for v in per.values()), default=0)}
json.dump(res, open(out, "w"), indent=1)
for c, r in res.items():
    k = r["counters"]
    print(c, r["kernel"], "MFMA busy per SIMD / GUI active per XCD: %.2f" %
          (k.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / max(k.get("GRBM_GUI_ACTIVE", 1) / 8, 1)))
