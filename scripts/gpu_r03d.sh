#!/bin/bash
# round 3: full GPU suite (scatter forward, multi-hot bwd prefetch, trajectory tests); TN stagger; stash arms
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03d}
mkdir -p $OUT
export TMPDIR=/tmp
export DLAMD_TEST_STATS=$OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in base tnstag; do
  if [ "$v" = base ]; then unset DLAMD_VARIANT; else export DLAMD_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "s3" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/s3test_$v.log 2>&1
  rc=$?; echo "s3 tests $v rc=$rc: $(tail -1 $OUT/s3test_$v.log)"; [ $rc -eq 0 ] || continue
  timeout -k 10 120 python scripts/s3_bench.py 20 > $OUT/s3bench_$v.txt 2>&1 || exit $?
  echo "== $v"; head -5 $OUT/s3bench_$v.txt
done
unset DLAMD_VARIANT
for arm in scat nostash scat2 idx; do
  extra=""; case $arm in nostash*) extra="--no-rec-stash";; esac
  [ $arm = idx ] && export DLAMD_FWD_SCATTER=0
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra $extra > $OUT/bench_$arm.json 2> $OUT/bench_$arm.err
  rc=$?; unset DLAMD_FWD_SCATTER; [ $rc -eq 0 ] || { echo "bench $arm rc=$rc"; tail -5 $OUT/bench_$arm.err; exit $rc; }
  python -c "
import json; d=json.load(open('$OUT/bench_$arm.json')); k=d['kernels']
print('$arm ms %.4f  bwd %.1f gather %.1f fwd %.1f' % (d['ms_per_step'], k['embed_bwd']['us'], k['rec_gather']['us'], k['embed_fwd']['us']))"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --workload c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
python -c "
import json; d=json.load(open('$OUT/bench_c3.json')); k=d['kernels']
print('c3 ms %.4f  bwd %.1f gather %.1f pool %.1f fwd %.1f' % (d['ms_per_step'], k['embed_bwd']['us'], k['rec_gather']['us'], k['pool_fwd']['us'], k['embed_fwd']['us']))"
