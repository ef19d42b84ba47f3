#!/bin/bash
# round 3: GPU suite + smoke + bench (no CPU baseline), scatter ubench, s3 NT read-ahead variants
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
export DLAMD_TEST_STATS=$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25 > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
cat $OUT/smoke.log
timeout -k 10 60 ./scripts/ubench_scatter.bin > $OUT/ubench_scatter.txt 2>&1 || exit $?
cat $OUT/ubench_scatter.txt
for v in base asmb1 asmb2 asmb3; do
  if [ "$v" = base ]; then unset DLAMD_VARIANT; else export DLAMD_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "s3" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/s3test_$v.log 2>&1
  rc=$?; echo "s3 tests $v rc=$rc: $(tail -1 $OUT/s3test_$v.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 120 python scripts/s3_bench.py 20 > $OUT/s3bench_$v.txt 2>&1 || exit $?
  echo "== $v"; cat $OUT/s3bench_$v.txt
done
unset DLAMD_VARIANT
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_default.json; exit $rc
