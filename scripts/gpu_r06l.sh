#!/bin/bash
# round 6: bf16 NT A-ring depth (DL_BN_PA 2 / 3 / 4): the bf16 GEMM tests on each variant, the
# bf16 GEMM bench, then C5 steps A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
for v in pa3 pa4; do
  DLAMD_VARIANT=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "bf16" > $O/pytest_$v.log 2>&1 || exit $?
done
for v in "" pa3 pa4 "" pa3 pa4; do
  DLAMD_VARIANT=$v timeout -k 10 200 python -u scripts/gemm_bf16_bench.py 20 2>/dev/null | grep -v amdgpu.ids | sed "s/^/[${v:-pa2}] /" >> $O/gemm_bf16.txt || exit $?
done
for v in "" pa3 pa4 "" pa3 pa4; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/c5_${v:-pa2}.log || exit $?
  grep "per-kernel\|ms/step" $O/c5_${v:-pa2}.log | tail -2 | sed "s/^/[${v:-pa2}] /" >> $O/ab.txt
done
