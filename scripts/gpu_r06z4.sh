#!/bin/bash
# round 6: the fused-gather parity tests after their refactor
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "gather or fused or lookup_without" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
