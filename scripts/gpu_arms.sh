#!/bin/bash
# Bench arms on one box, each arm an environment (DLAMD_VARIANT=..., DL_...=...), after an
# optional focused pytest selection; prints per arm the step, the gather pair and lookup alone.
#   bash scripts/gpu_arms.sh TAG "<pytest -k or empty>" "<workloads>" "label=ENV[,ENV...]" ...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf -k "$2" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
WLS=$3; shift 3
for rep in 1 2; do
  for wl in $WLS; do
    for arm in "$@"; do
      label=${arm%%=*}; envs=${arm#*=}; E=${envs//,/ }
      [ "$envs" = "$arm" ] && E=""
      f=$OUT/bench_${wl}_${label}_$rep
      env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "
import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);k=d['kernels'];g=d.get('gather_north_star') or {}
la=g.get('lookup_alone') or {}
print('$wl $label', d['ms_per_step'], 'pair', g.get('us'), 'alone', la.get('us'), 'zipf', (la.get('zipf') or {}).get('us'),
      {n: k[n]['us'] for n in k if k[n]['us'] >= 40})" | tee -a $OUT/arms.txt
    done
  done
done
