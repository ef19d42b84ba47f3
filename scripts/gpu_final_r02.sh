#!/bin/bash
# round-2 close: GPU suite, smoke, fwd-bound A/B (base vs fwdold), rocprofv3 kernel stats of the default bench
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -8 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_default.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_variants.sh r02u/ab base fwdold || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o trace -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"
exit $rc
