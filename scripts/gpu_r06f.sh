#!/bin/bash
# round 6: wdl head prefetch A/B (C5), the wdl GPU tests, the HBM copy yardstick, the default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dropin.py -k "wdl" > $O/pytest_wdl.log 2>&1 || exit $?
for v in "" headold "" headold; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 >> $O/c5_${v:-new}.json 2>> $O/c5_${v:-new}.log || exit $?
done
timeout -k 10 120 python -u scripts/hbm_copy_bench.py > $O/hbm_copy.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log
