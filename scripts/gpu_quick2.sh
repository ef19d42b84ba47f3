#!/bin/bash
# targeted GPU tests + C2/C3 bench. Usage: bash scripts/gpu_quick2.sh TAG "pytest -k expr"
TAG=${1:-q2}; K=${2:-"lazy or multi or pool"}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider -x -k "$K" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for W in c2 c3; do
  timeout -k 10 600 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$W.json 2> $OUT/bench_$W.err
  rc=$?; echo "bench $W rc=$rc"; python -c "import json,sys; d=json.load(open('$OUT/bench_$W.json')); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items() if v['us'] > 90})"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
