#!/bin/bash
# A/B session: focused GPU tests, then the given benches. bash scripts/gpu_ab.sh TAG "<pytest -k>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT; K=$2
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$K" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
for v in "" rs32; do
  for wl in c2 c3; do
    DLAMD_VARIANT=$v timeout -k 10 120 python scripts/index_bench.py $wl 20 2>&1 | grep -v amdgpu.ids | sed "s/^/${v:-base} /" || exit 1
  done
done
timeout -k 10 120 python scripts/s3_bench.py 20 > $OUT/s3bench.txt 2>&1 || exit $?
grep -v amdgpu.ids $OUT/s3bench.txt | head -8
for arm in bits f32mask; do
  [ $arm = f32mask ] && export DLAMD_RELU_BITS=0
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $OUT/bench_$arm.json 2> $OUT/bench_$arm.err || { tail -5 $OUT/bench_$arm.err; exit 1; }
  unset DLAMD_RELU_BITS
  echo "== $arm"; python scripts/bench_brief.py $OUT/bench_$arm.json
done
