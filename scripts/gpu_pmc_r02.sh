#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter set per run) over the default C2 bench,
# for profiles/<TAG>/pmc_summary.json (scripts/pmc_summary.py). Usage: bash scripts/gpu_pmc_r02.sh TAG
TAG=${1:-r02s}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o trace -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o fetch -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_fetch.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o write -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_write.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_summary.py $OUT $OUT/pmc_summary.json && echo summary ok
