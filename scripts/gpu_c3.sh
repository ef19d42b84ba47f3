#!/bin/bash
# multi-hot records bring-up: lazy/multi parity tests, then C3 bench dense vs lazy. Usage: bash scripts/gpu_c3.sh TAG
TAG=${1:-c3}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "lazy or multi" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for A in lazy dense; do
  timeout -k 10 600 python bench.py --workload c3 --adam $A --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c3_$A.json 2> $OUT/bench_c3_$A.err
  rc=$?; echo "bench c3 $A rc=$rc"; tail -3 $OUT/bench_c3_$A.err; cat $OUT/bench_c3_$A.json
  if [ $rc -ne 0 ]; then exit $rc; fi
done
