#!/bin/bash
# round 6: the bf16 tower's ReLU sign bitmask (dl_gemm_bf16_bits): kernel tests, the wdl / bf16
# parity and shard tests, then C5 A/B (DLAMD_RELU_BITS=0: the bf16 activations as the mask)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_shard.py -k "bf16 or wdl" > $O/pytest.log 2>&1 || exit $?
tail -2 $O/pytest.log
for a in 1 0 1 0; do
  DLAMD_RELU_BITS=$a timeout -k 10 300 python -u bench.py --workload c5 --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/c5_$a.log || exit $?
  grep "ms/step\|per-kernel" $O/c5_$a.log | tail -2 | sed "s/^/[bits=$a] /" >> $O/ab.txt
done
