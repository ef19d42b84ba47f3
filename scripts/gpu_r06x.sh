#!/bin/bash
# round 6: the s3 dX bitmask words loaded before the last k step (default) against before the
# main loop (variant mwearly: 7 spilled VGPRs): s3 tests, then C2 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "s3 or relu_bitmask or deepfm_pipeline or fp64" > $O/pytest.log 2>&1 || exit $?
tail -2 $O/pytest.log
for v in "" mwearly "" mwearly; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/c2_${v:-main}.log || exit $?
  grep "headline" $O/c2_${v:-main}.log | tail -1 | cut -c1-420 | sed "s/^/[${v:-main}] /" >> $O/ab.txt
done
