#!/bin/bash
# A/B session: focused GPU tests, then bench arms. bash scripts/gpu_ab.sh TAG "<pytest -k>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT; K=$2
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$K" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
run() {   # run NAME ENV... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; return 1; }
  echo "== $name $(python -c "import json;d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items() if k.startswith('gemm')})")"
}
for v in "" bnd2; do
  DLAMD_VARIANT=$v timeout -k 10 120 python scripts/gemm_bf16_bench.py 20 > $OUT/bf16bench_${v:-d4}.txt 2>&1 || exit 1
  echo "== bf16 ${v:-d4}"; grep -v amdgpu.ids $OUT/bf16bench_${v:-d4}.txt | head -3
done
run c5_d4 DLAMD_VARIANT= -- --workload c5 --steps 20 --warmup 5 || exit 1
run c5_d2 DLAMD_VARIANT=bnd2 -- --workload c5 --steps 20 --warmup 5 || exit 1
