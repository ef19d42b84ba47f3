#!/bin/bash
# The north-star lookup alone, uniform and Zipf ids: time, rocprofv3 stats, FETCH / WRITE / L2
# hit passes (one counter set a run), then the random 64-B gather microbenchmark on the same
# box as the access-pattern ceiling: bash scripts/gpu_lookup_pmc.sh TAG [full|fm]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${1:-lk}; MODE=${2:-full}; mkdir -p $OUT
for d in uniform zipf; do
  timeout -k 10 200 python scripts/lookup_bench.py $d 20 $MODE > $OUT/lookup_$d.txt 2>&1 || { tail -5 $OUT/lookup_$d.txt; exit 1; }
  grep lookup $OUT/lookup_$d.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/st_$d -o t -- python scripts/lookup_bench.py $d 20 $MODE > /dev/null 2>&1 || { echo "stats $d failed"; exit 1; }
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${d}_$i -o p -- python scripts/lookup_bench.py $d 5 $MODE > /dev/null 2>&1 || { echo "pmc $d pass $i failed"; exit 1; }
  done
done
python - <<PY
import csv, glob, json
out = {}
KEEP = ("embed_fwd", "gemm_s3_nt")
def short(n):
    return n.split("(")[0].replace("void ", "").replace("dl::", "")[:60]
for d in ("uniform", "zipf"):
    r = {}
    f = glob.glob("$OUT/st_%s/**/t_kernel_stats.csv" % d, recursive=True)[0]
    for row in csv.DictReader(open(f)):
        if any(k in row["Name"] for k in KEEP):
            r.setdefault(short(row["Name"]), {}).update(avg_us=float(row["AverageNs"]) / 1e3, calls=int(row["Calls"]))
    ctr = {}
    for f in glob.glob("$OUT/pmc_%s_*/**/p_counter_collection.csv" % d, recursive=True):
        for row in csv.DictReader(open(f)):
            if not any(k in row["Kernel_Name"] for k in KEEP):
                continue
            key = (short(row["Kernel_Name"]), row["Counter_Name"], f, row["Dispatch_Id"])
            ctr[key] = ctr.get(key, 0.0) + float(row["Counter_Value"])   # summed over instances
    per = {}
    for (kn, name, _, _), v in ctr.items():
        per.setdefault(kn, {}).setdefault(name, []).append(v)
    for kn, cs in per.items():
        r.setdefault(kn, {})["counters_per_launch"] = {k: sum(v) / len(v) for k, v in cs.items()}
    out[d] = r
json.dump(out, open("$OUT/lookup_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
hipcc -O3 --offload-arch=gfx950 scripts/ubench_gather.hip -o /tmp/ubench_gather && timeout -k 10 120 /tmp/ubench_gather > $OUT/ubench_gather_26M.txt 2>&1; cat $OUT/ubench_gather_26M.txt
