#!/bin/bash
# round 6: bf16 NT kernel (hand-counted A waits, 16-B bf16 stores) vs bnold; m-only stash vs stash0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
for v in "" bnold; do
  DLAMD_VARIANT=$v timeout -k 10 120 python -u scripts/gemm_bf16_bench.py 50 > $O/gemm_bf16_${v:-new}.txt 2>&1 || exit $?
done
for v in "" bnold "" bnold; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 >> $O/c5_${v:-new}.json 2>> $O/c5_${v:-new}.log || exit $?
done
for v in "" stash0 "" stash0; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c2 --no-extra --no-cpu-baseline --steps 30 >> $O/c2_${v:-new}.json 2>> $O/c2_${v:-new}.log || exit $?
done
timeout -k 10 120 python -u scripts/hbm_copy_bench.py > $O/hbm_copy.txt 2>&1
