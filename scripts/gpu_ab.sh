#!/bin/bash
# A/B session: focused GPU tests, then bench arms. bash scripts/gpu_ab.sh TAG "<pytest -k>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT; K=$2
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -k "$K" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
run() {   # run NAME ENV... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; return 1; }
  echo "== $name $(python -c "import json;d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]);k=d['kernels'];print(d['ms_per_step'], {n: k[n]['us'] for n in ('head', 'wide_grad', 'adam_wide', 'index_build', 'index_build_wide') if n in k})")"
}
run c5 -- --workload c5 --steps 20 --warmup 5 || exit 1
run c3 -- --workload c3 --steps 10 --warmup 3 || exit 1
run c2 -- --steps 30 --warmup 5 || exit 1
