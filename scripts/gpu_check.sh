#!/bin/bash
# Whole GPU suite + C5 and C2 bench lines (no CPU baseline): bash scripts/gpu_check.sh TAG
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${1:-check}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=5 > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.log | head -20; exit $rc; }
for wl in c5 c2 c3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -5 $OUT/bench_$wl.err; exit 1; }
  python -c "
import json;d=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$wl', d['ms_per_step'], {n: k[n]['us'] for n in k})"
done
