#!/bin/bash
# round 6, first GPU call: the tests this round's changes touch, the GEMM yardstick, the default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dropin.py tests/test_gpu_kernels.py::test_adam_rows_width1_sweep \
  tests/test_shard.py::test_sharded_all_reduce_placement_equals_global_batch \
  tests/test_shard.py::test_sharded_bad_id_on_one_rank_raises_everywhere \
  "tests/test_shard.py::test_sharded_engine_two_ranks_equals_global_batch" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_yardstick.py 20 > $O/gemm_yardstick.json 2> $O/gemm_yardstick.log || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log
