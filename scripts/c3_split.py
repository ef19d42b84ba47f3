"""C3's HBM bytes by access stream (scripts/gpu_r06e.sh): per kernel, FETCH_SIZE and WRITE_SIZE
(bytes per dispatch, mean over the dispatches) of the default build and of each diagnostics build
that redirects one stream to a cache-resident address; a stream's bytes are the default's minus
the diagnostics build's.  FETCH deltas are given raw and with gfx950's x2 correction (coalesced
streaming reads are tallied at half their bytes, MI355X_MICROARCH.md; a random 64-B request is
tallied whole, profiles/r04g/bwd_split.json) — random streams are read raw.
    python scripts/c3_split.py gpurun_out/r06e profiles/r06e/c3_split.json"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

VARIANTS = {
    "bd1": ("rec_bwd_adam", "dx0 slices of the single deep references (random 64 B)"),
    "bd2": ("rec_bwd_adam", "fm_sum rows of the FM references (random 64 B)"),
    "bd4": ("rec_bwd_adam", "stash + compact rows (sequential, u order)"),
    "bd8": ("rec_bwd_adam", "record writes (256 B, whole lines)"),
    "bd16": ("rec_bwd_adam", "pooled-slot gradients of the multi-hot references (random 64 B)"),
    "pd1": ("pool_fwd", "compact rows of the multi-hot positions (random 64 B)"),
    "pd2": ("pool_fwd", "pooled / count / first-order outputs"),
    "pw": ("pool_fwd", "first-order weights of the multi-hot positions (random 4 B)"),
}


def short(n):
    n = re.sub(r"\(.*$", "", n)
    return re.sub(r"^void ", "", n).replace("dl::", "")


def per_kernel(d):
    out = defaultdict(dict)
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(d, ctr + "_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
        for k, v in acc.items():
            out[k][ctr] = sum(v) / len(v)
    return out


def find(runs, key):
    return next((k for k in runs if k.startswith(key)), None)


def main(src, dst):
    base = per_kernel(os.path.join(src, "new"))
    res = {"note": __doc__.split("\n\n")[0], "kernels": {}}
    for kk in ("rec_bwd_adam", "pool_fwd"):
        k = find(base, kk + "_kernel") or find(base, kk)
        if k is None:
            continue
        b = base[k]
        ent = {"kernel": k, "fetch_raw": b.get("FETCH_SIZE"), "write": b.get("WRITE_SIZE"), "streams": {}}
        for v, (target, what) in VARIANTS.items():
            if target != kk:
                continue
            r = per_kernel(os.path.join(src, v))
            rk = find(r, kk + "_kernel") or find(r, kk)
            if rk is None:
                continue
            ent["streams"][what] = {"variant": v, "fetch_raw_delta": b.get("FETCH_SIZE", 0) - r[rk].get("FETCH_SIZE", 0),
                                    "write_delta": b.get("WRITE_SIZE", 0) - r[rk].get("WRITE_SIZE", 0)}
        rnd = sum(s["fetch_raw_delta"] for n, s in ent["streams"].items() if "random" in n)
        ent["hbm_bytes_x2_everywhere"] = 2 * b.get("FETCH_SIZE", 0) + b.get("WRITE_SIZE", 0)
        ent["hbm_bytes_calibrated"] = 2 * (b.get("FETCH_SIZE", 0) - rnd) + rnd + b.get("WRITE_SIZE", 0)
        res["kernels"][kk] = ent
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
