#!/bin/bash
# hipGraph replay vs eager launches, single GPU and one-rank sharded; sharded trace.
TAG=${1:-gab}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for V in "" "--no-graph" "--sharded" "--sharded --no-graph"; do
  N=$(echo "x$V" | tr -d ' -')
  timeout -k 10 600 python bench.py $V --steps 30 --warmup 5 --no-cpu-baseline > $OUT/b_$N.json 2> $OUT/b_$N.err
  rc=$?; echo "bench [$V] rc=$rc"; python -c "import json; d=json.load(open('$OUT/b_$N.json')); print(d['value'], d['ms_per_step'])"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python bench.py --sharded --steps 6 --warmup 3 --no-cpu-baseline > $OUT/tr.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
