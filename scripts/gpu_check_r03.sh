#!/bin/bash
# round-3 check: GPU suite, smoke, default bench. Usage: bash scripts/gpu_check_r03.sh <tag>
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
export TMPDIR=/tmp
export DLAMD_TEST_STATS=$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25 > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_default.json; exit $rc
