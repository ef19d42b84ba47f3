#!/bin/bash
# Per-kernel split of the batch index build alone (rocprofv3 --kernel-trace --stats) at C2 and C3,
# for the default library and optionally a variant: bash scripts/gpu_index_prof.sh TAG [VARIANT]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${1:-idx}; mkdir -p $OUT
for v in "" $2; do
for wl in c2 c3; do
  D=$OUT/${v:-new}_$wl
  DLAMD_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- python scripts/index_bench.py $wl 20 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  echo "== ${v:-new} $(grep index_build $D.log)"
  python - <<PY
import csv, glob
f = glob.glob("$D/**/t_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("rs_", "unique", "index", "validate", "keys")):
        print("  %-34s calls %5s avg %8.1f us" % (n[:34], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
done
