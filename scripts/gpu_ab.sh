#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "bf16 or wdl or gemm" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
for v in "" bres; do
  DLAMD_VARIANT=$v timeout -k 10 120 python scripts/gemm_bf16_bench.py 20 > $OUT/bf16bench_${v:-nt}.txt 2>&1 || exit $?
  echo "== bf16 ${v:-nt}"; cat $OUT/bf16bench_${v:-nt}.txt | grep -v amdgpu.ids
done
for v in "" nosplit nostore; do
  DLAMD_VARIANT=$v timeout -k 10 120 python scripts/s3_bench.py 20 > $OUT/s3bench_${v:-base}.txt 2>&1 || exit $?
  echo "== s3 ${v:-base}"; grep -v amdgpu.ids $OUT/s3bench_${v:-base}.txt | head -6
done
for wl in c5 c3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 10 --warmup 3 > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -5 $OUT/bench_$wl.err; exit 1; }
  python scripts/bench_brief.py $OUT/bench_$wl.json
done
