#!/bin/bash
# GPU check + bench + rocprofv3 evidence. Usage: bash scripts/gpu_profile.sh TAG [bench args...]
TAG=${1:-run}; shift
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "(tests run separately)"


timeout -k 10 600 python bench.py --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o trace -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $OUT/prof_trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o fetch -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/prof_fetch.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o write -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/prof_write.log 2>&1
rc=$?; echo "rocprof write rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
