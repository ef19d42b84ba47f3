#!/bin/bash
# round 6: C3 HBM bytes by access stream — FETCH_SIZE / WRITE_SIZE passes over the default build
# and the diagnostics builds that redirect one stream (DL_BWD_DIAG 1/2/4/8/16, DL_POOL_DIAG 1/2,
# DL_POOL_DIAG_NO_W1), one rocprofv3 run a pass; plus the step's time per build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
for v in new bd1 bd2 bd4 bd8 bd16 pd1 pd2 pw; do
  V=$v; [ $v = new ] && V=""
  for ctr in FETCH_SIZE WRITE_SIZE; do
    DLAMD_VARIANT=$V timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/$v -o ${ctr} --output-format csv -- python scripts/c3_steps.py 6 24 > $O/${v}_${ctr}.log 2>&1 || { echo "pmc $v $ctr failed"; exit 1; }
  done
  echo "$v done"
done
# the 4-wave (128-row) register-epilogue bf16 NT blocks against the 8-wave default
DLAMD_VARIANT=nw4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "bf16" > $O/pytest_nw4_bf16.log 2>&1 || exit $?
for v in "" nw4; do
  DLAMD_VARIANT=$v timeout -k 10 120 python -u scripts/gemm_bf16_bench.py 50 > $O/gemm_bf16_${v:-new}.txt 2>&1 || exit $?
done
for v in "" nw4 "" nw4; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 >> $O/c5_${v:-new}.json 2>> $O/c5_${v:-new}.log || exit $?
done
timeout -k 10 120 python -u scripts/hbm_copy_bench.py > $O/hbm_copy.txt 2>&1
