#!/bin/bash
# A/B of the default library against an experiment variant (libdlamd_<VAR>.so, built with
# DLAMD_VARIANT=<VAR> DLAMD_DEFINES=...): focused tests, a microbench script, then bench arms.
#   bash scripts/gpu_ab_variant.sh TAG VAR "<pytest -k>" "<ubench script + args>" "<workloads>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; VAR=$2; mkdir -p $OUT
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$3" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
if [ -n "$4" ]; then
  timeout -k 10 200 python $4 > $OUT/ubench_new.txt 2>&1 || exit $?
  DLAMD_VARIANT=$VAR timeout -k 10 200 python $4 > $OUT/ubench_$VAR.txt 2>&1 || exit $?
  echo "== new"; grep -v amdgpu.ids $OUT/ubench_new.txt; echo "== $VAR"; grep -v amdgpu.ids $OUT/ubench_$VAR.txt
fi
for wl in $5; do
  for arm in new $VAR new $VAR; do
    if [ $arm = new ]; then E=""; else E="DLAMD_VARIANT=$VAR"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 > $OUT/bench_${wl}_$arm.json 2> $OUT/bench_${wl}_$arm.err || { tail -5 $OUT/bench_${wl}_$arm.err; exit 1; }
    python -c "
import json;d=json.loads(open('$OUT/bench_${wl}_$arm.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$wl $arm', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'), {n: k[n]['us'] for n in k if k[n]['us'] >= 30})"
  done
done
