#!/bin/bash
# selected GPU tests ($1: pytest -k expression or "none"), then the default bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$1" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 600 --timeout-method thread -k "$1" > gpurun_out/pytest_sel.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; tail -8 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
