cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r03dw; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -rf -k "bf16_dw" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_dw.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_dw.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $OUT/pytest_dw.log | head -20; exit $rc; }
timeout -k 10 120 python scripts/gemm_bf16_bench.py 20 > $OUT/ubench_new.txt 2>&1 || exit $?
DLAMD_VARIANT=olddw timeout -k 10 120 python scripts/gemm_bf16_bench.py 20 > $OUT/ubench_old.txt 2>&1 || exit $?
echo NEW; cat $OUT/ubench_new.txt; echo OLD; cat $OUT/ubench_old.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload c5 --steps 20 --warmup 5 > $OUT/bench_c5_new.json 2> $OUT/bench_c5_new.err || { tail -5 $OUT/bench_c5_new.err; exit 1; }
DLAMD_VARIANT=olddw DLAMD_DW_SPLITS=64 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload c5 --steps 20 --warmup 5 > $OUT/bench_c5_old.json 2> $OUT/bench_c5_old.err || { tail -5 $OUT/bench_c5_old.err; exit 1; }
for a in new old; do python -c "
import json;d=json.loads(open('$OUT/bench_c5_$a.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$a', d['ms_per_step'], {n: k[n]['us'] for n in k if 'dw' in n or 'adam_dense' in n})"; done
