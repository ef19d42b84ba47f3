#!/bin/bash
# A/B of an engine environment switch: focused tests, then bench arms with and without it.
#   bash scripts/gpu_ab_env.sh TAG "VAR=VALUE" "<pytest -k>" "<workloads>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; EV=$2; mkdir -p $OUT
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$3" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
for wl in $4; do
  for arm in new old new old; do
    if [ $arm = new ]; then E="DLAMD_AB_ARM=new"; else E="$EV"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 > $OUT/bench_${wl}_$arm.json 2> $OUT/bench_${wl}_$arm.err || { tail -5 $OUT/bench_${wl}_$arm.err; exit 1; }
    python -c "
import json;d=json.loads(open('$OUT/bench_${wl}_$arm.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$wl $arm', d['ms_per_step'], {n: k[n]['us'] for n in k if 'gemm' not in n and 'adam' not in n})"
  done
done
