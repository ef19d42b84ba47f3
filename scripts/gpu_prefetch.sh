#!/bin/bash
# prefetch parity + C2/C3 bench with and without prefetch.
TAG=${1:-pf}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "prefetch or lazy or graph" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for V in "" "--no-prefetch" "--workload c3" "--workload c3 --no-prefetch" "--workload c5"; do
  N=$(echo "x$V" | tr -d ' -')
  timeout -k 10 600 python bench.py $V --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b_$N.json 2> $OUT/b_$N.err
  rc=$?; echo "bench [$V] rc=$rc"; python -c "import json; d=json.load(open('$OUT/b_$N.json')); print(d['value'], d['ms_per_step'])"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline > $OUT/tr.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
