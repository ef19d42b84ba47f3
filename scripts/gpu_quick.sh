#!/bin/bash
# quick GPU iteration: tests + bench. Usage: bash scripts/gpu_quick.sh TAG [bench args...]
TAG=${1:-quick}; shift
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.err; cat $OUT/bench.json; exit $rc
