"""The backward's HBM bytes split by access stream (scripts/gpu_r4.sh bwddiag): FETCH_SIZE /
WRITE_SIZE of rec_bwd_adam for the default build and the DL_BWD_DIAG builds that redirect one
stream to a cache-resident address (d1: the dx0 slices, d2: the fm_sum rows, d8: no record
writes).  Each stream's raw FETCH_SIZE delta is reported with the gfx950 x2 correction
(MI355X_MICROARCH.md: coalesced streaming reads are tallied at half their bytes) and without:
a random 64-B slice read is one 64-B request, so its raw delta already is its byte count.

    python scripts/bwd_split.py gpurun_out/r04g profiles/r04g/bwd_split.json
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*$", "", n)
    return re.sub(r"^void ", "", n).replace("dl::", "")


def counters(d):
    res = {}
    for ctr, sub in (("FETCH_SIZE", "prof_fetch/fetch_counter_collection.csv"),
                     ("WRITE_SIZE", "prof_write/write_counter_collection.csv")):
        acc = defaultdict(list)
        for r in csv.DictReader(open("%s/%s" % (d, sub))):
            if r["Counter_Name"] == ctr:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            res.setdefault(k, {})[ctr] = sum(v) / len(v) * 1024   # bytes per dispatch
    return res


def main(src, dst):
    runs = {v: counters("%s/bwd_%s" % (src, v)) for v in ("new", "d1", "d2", "d8")}
    k = next(n for n in runs["new"] if n.startswith("rec_bwd_adam_kernel"))
    base = runs["new"][k]
    out = {"kernel": k, "raw_fetch_bytes": base["FETCH_SIZE"], "write_bytes": base["WRITE_SIZE"], "streams": {}}
    for v, what in (("d1", "dx0 slices (random 64 B)"), ("d2", "fm_sum rows (random 64 B, 4.2 MB reused 26x)"),
                    ("d8", "record writes (256 B, whole lines)")):
        r = runs[v][k]
        out["streams"][what] = {"raw_fetch_delta": base["FETCH_SIZE"] - r["FETCH_SIZE"],
                                "write_delta": base["WRITE_SIZE"] - r["WRITE_SIZE"]}
    rnd = sum(s["raw_fetch_delta"] for n, s in out["streams"].items() if "random" in n)
    out["hbm_bytes_x2_everywhere"] = 2 * base["FETCH_SIZE"] + base["WRITE_SIZE"]
    out["hbm_bytes_calibrated"] = 2 * (base["FETCH_SIZE"] - rnd) + rnd + base["WRITE_SIZE"]
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
