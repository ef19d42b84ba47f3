#!/bin/bash
# The round's GPU evidence, in two calls (each under gpurun's limit):
#   bash scripts/gpu_round.sh suite TAG   full `pytest -m gpu` (+ measured stats), smoke(), default bench
#   bash scripts/gpu_round.sh prof TAG    per workload (c2, c3, c5): rocprofv3 --kernel-trace --stats and
#                                         separate FETCH_SIZE / WRITE_SIZE passes -> pmc_summary_<wl>.json;
#                                         SQ counter passes over the s3 GEMM cases
# Results land in gpurun_out/TAG; the judged copies go to profiles/TAG.
MODE=$1
TAG=${2:-run}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

if [ "$MODE" = suite ]; then
  export DLAMD_TEST_STATS=$OUT
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
    --durations=15 > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  unset DLAMD_TEST_STATS
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_default.err; exit $rc; }
  python scripts/bench_brief.py $OUT/bench_default.json
  exit 0
fi

if [ "$MODE" = prof ]; then
  for wl in c2 c3 c5; do
    W=$OUT/$wl
    mkdir -p $W
    args="--no-cpu-baseline --no-extra --workload $wl"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/prof_trace -o trace -- \
      python bench.py --steps 10 --warmup 3 $args > $W/prof_trace.log 2>&1
    rc=$?; echo "$wl trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $W/prof_fetch -o fetch -- \
      python bench.py --steps 3 --warmup 1 $args > $W/prof_fetch.log 2>&1
    rc=$?; echo "$wl fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $W/prof_write -o write -- \
      python bench.py --steps 3 --warmup 1 $args > $W/prof_write.log 2>&1
    rc=$?; echo "$wl write rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python scripts/pmc_summary.py $W $OUT/pmc_summary_$wl.json $wl > $W/summary.txt && head -12 $W/summary.txt
  done
  bash scripts/pmc_s3.sh $OUT/s3pmc fwd_l1 dw_l1 || exit $?
  python scripts/sq_summary.py $OUT/s3pmc $OUT/s3_sq_counters.json fwd_l1 dw_l1
  exit 0
fi
if [ "$MODE" = rehearse ]; then
  # the multi-rank bench flow on one GPU: bench.py --gpus 2 starts its two ranks itself
  # (gloo-staged exchange, both ranks on device 0), then the same under the driver's launcher form
  DLAMD_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 --age-steps 8 \
    --extra-steps 3 > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err
  rc=$?; echo "bench --gpus 2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_gpus2.err; exit $rc; }
  python scripts/bench_brief.py $OUT/bench_gpus2.json
  exit 0
fi
echo "usage: gpu_round.sh suite|prof|rehearse TAG"; exit 2
