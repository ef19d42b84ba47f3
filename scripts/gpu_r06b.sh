#!/bin/bash
# round 6: the bf16 NT kernel with hand-counted A waits + 16-B bf16 stores, against the old build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "bf16" > $O/pytest_bf16.log 2>&1 || exit $?
for v in "" bnold; do
  DLAMD_VARIANT=$v timeout -k 10 120 python -u scripts/gemm_bf16_bench.py 50 > $O/gemm_bf16_${v:-new}.txt 2>&1 || exit $?
done
for v in "" bnold "" bnold; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 > $O/c5_${v:-new}.json 2>> $O/c5_${v:-new}.log || exit $?
done
timeout -k 10 120 python -u scripts/hbm_copy_bench.py > $O/hbm_copy.txt 2>&1
