#!/bin/bash
# Round-5 GPU session: steps named on the command line, each under its own time limit; a
# step that times out, aborts or faults (rc >= 124) ends the session, a failing test does not.
#   bash scripts/gpu_r05.sh TAG step [step ...]
#   steps: shard | gemm_epd | kernels | parity | fullsize | bench | benchsh | smoke | all_gpu
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; shift; mkdir -p $OUT
run() {   # run NAME LIMIT CMD...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "[$name] rc=$rc $(grep -v amdgpu.ids $OUT/$name.log | tail -1)"
  if [ $rc -ge 124 ]; then echo "[$name] stopping the session (rc $rc)"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  case $step in
    shard) run shard 700 $PYT tests/test_gpu_shard.py tests/test_shard.py -m gpu ;;
    kernels) run kernels 900 $PYT tests/test_gpu_kernels.py tests/test_gpu_comm.py -m gpu ;;
    parity) run parity 1100 env DLAMD_TEST_STATS=$OUT $PYT tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu ;;
    fullsize) run fullsize 1150 env DLAMD_TEST_STATS=$OUT $PYT tests/test_gpu_fullsize.py -m gpu ;;
    all_gpu) run all_gpu 1150 env DLAMD_TEST_STATS=$OUT $PYT tests -m gpu ;;
    c1) run c1 600 env DLAMD_TEST_STATS=$OUT $PYT tests/test_gpu_parity.py -m gpu -k "c1_defaults or bf16_tower" ;;
    suite) run suite 1100 env DLAMD_TEST_STATS=$OUT $PYT tests -m gpu --ignore=tests/test_gpu_fullsize.py ;;
    gemm_ab_*)   # gemm_ab_<variant>: GEMM tests on the variant, s3_bench and C2 A/B
      v=${step#gemm_ab_}
      run ${v}_tests 600 env DLAMD_VARIANT=$v $PYT tests/test_gpu_kernels.py -m gpu -k "s3 or gemm"
      for a in base $v base $v; do
        if [ $a = base ]; then E=""; else E=$a; fi
        run s3_$a 200 env DLAMD_VARIANT=$E python scripts/s3_bench.py 20
        grep -v amdgpu.ids $OUT/s3_$a.log | sed "s/^/[$a] /" >> $OUT/s3_ab.txt
      done
      for a in base $v base $v; do
        if [ $a = base ]; then E=""; else E=$a; fi
        run c2_$a 300 env DLAMD_VARIANT=$E python bench.py --no-cpu-baseline --no-extra --steps 20
        grep '^{' $OUT/c2_$a.log | python -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);k=d['kernels']
print('$a', d['ms_per_step'], {n: k[n]['us'] for n in k if n.startswith('gemm')})" >> $OUT/c2_ab.txt
      done ;;
    envab_*)   # envab_<VAR>_<workload>[_<dist>]: bench arms VAR=0 / 1 / 0 / 1 on one box
      rest=${step#envab_}; var=${rest%%__*}; wl=${rest#*__}; dist=uniform
      case $wl in *_zipf) dist=zipf; wl=${wl%_zipf} ;; esac
      for a in 0 1 0 1; do
        run ${var}_${wl}_${dist}_$a 300 env $var=$a python bench.py --workload $wl --dist $dist --no-cpu-baseline --no-extra --steps 20
        grep '^{' $OUT/${var}_${wl}_${dist}_$a.log | python -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);k=d['kernels']
print('$var=$a $wl $dist', d['ms_per_step'], {n: k[n]['us'] for n in k})" >> $OUT/envab.txt
      done ;;
    s3env_*)   # s3env_<VAR>: the s3 / GEMM kernel tests with VAR=1, then s3_bench VAR=0 / 1 / 0 / 1
      var=${step#s3env_}
      run ${var}_tests 600 env $var=1 $PYT tests/test_gpu_kernels.py -m gpu -k "s3"
      for a in 0 1 0 1; do
        run s3_${var}_$a 200 env $var=$a python scripts/s3_bench.py 20
        grep -v amdgpu.ids $OUT/s3_${var}_$a.log | sed "s/^/[$var=$a] /" >> $OUT/s3_ab.txt
      done ;;
    bf16pmc)   # counters of the C5 tower's bf16 NT products (gemm_bf16_bench cases)
      run bf16pmc 600 bash scripts/pmc_bf16.sh $OUT/bf16pmc "fwd_l0 bf16 out relu" "dx_l1 mask bf16" &&
      SQ_KERNEL=gemm_bf16 python scripts/sq_summary.py $OUT/bf16pmc $OUT/bf16_sq_counters.json \
        fwd_l0_bf16_out_relu dx_l1_mask_bf16 > $OUT/bf16_sq.txt 2>&1
      run bf16bench 200 python scripts/gemm_bf16_bench.py 20 ;;
    tests_*)   # tests_<pattern>: the GPU tests whose names match
      run tests_sel 900 $PYT tests -m gpu -k "${step#tests_}" ;;
    bench) run bench 900 python bench.py ;;
    benchsh) run benchsh 600 python bench.py --sharded --no-extra --no-cpu-baseline --steps 20 ;;
    benchsh_c2) run benchsh_c2 600 python bench.py --sharded --no-extra --no-cpu-baseline --steps 20 --vocab 1000000 ;;
    benchc2) run benchc2 600 python bench.py --no-extra --no-cpu-baseline --steps 20 ;;
    benchc4single) run benchc4single 600 python bench.py --no-extra --no-cpu-baseline --steps 20 --vocab 3846154 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step" ;;
  esac
done
