#!/bin/bash
# C3 (multi-hot, lazy) parity subset + bench + kernel-trace profile. Usage: bash scripts/gpu_c3_prof.sh TAG
TAG=${1:-c3p}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "lazy or multi" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_c3.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; find $OUT/prof -name "*kernel_stats.csv" | head -3
