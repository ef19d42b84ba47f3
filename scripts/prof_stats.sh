#!/bin/bash
# rocprofv3 kernel stats of one command: bash scripts/prof_stats.sh TAG python script.py args...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o k -- "$@" > $OUT/prof.log 2>&1
rc=$?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(r["Name"][:70].ljust(70), r["Calls"].rjust(6), "%9.1f us" % (float(r["AverageNs"]) / 1e3))
PY
exit $rc
