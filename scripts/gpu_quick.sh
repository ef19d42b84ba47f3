#!/bin/bash
# A focused GPU check: bash scripts/gpu_quick.sh TAG "<pytest -k expr>" [bench args...]
# (the -k subset of the GPU suite, then one bench run with the given args)
TAG=$1; K=$2; shift 2
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$K" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python scripts/bench_brief.py $OUT/bench.json
