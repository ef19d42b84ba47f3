#!/bin/bash
# lazy-Adam bring-up: targeted tests, then dense vs lazy bench. Usage: bash scripts/gpu_lazy.sh TAG
TAG=${1:-lazy}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "lazy" > $OUT/pytest_lazy.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/pytest_lazy.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --adam lazy > $OUT/bench_lazy.json 2> $OUT/bench_lazy.err
rc=$?; echo "bench lazy rc=$rc"; tail -3 $OUT/bench_lazy.err; cat $OUT/bench_lazy.json; exit $rc
