#!/bin/bash
# one-rank sharded (RCCL) bench + kernel trace for the step timeline. Usage: bash scripts/gpu_shard_trace.sh TAG
TAG=${1:-shtr}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python bench.py --sharded --steps 6 --warmup 3 --no-cpu-baseline > $OUT/tr.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
