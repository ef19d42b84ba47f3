#!/bin/bash
# sharded path: GPU tests (2 gloo ranks on one GPU) + parity subset, one-rank RCCL bench, trace.
TAG=${1:-shc}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_shard.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider -x -k "shard or sorted or lazy or chain" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items() if v['us'] > 90})"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err
rc=$?; echo "bench c2 rc=$rc"; python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print(d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['kernels'].items() if v['us'] > 90})"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python bench.py --sharded --steps 6 --warmup 3 --no-cpu-baseline > $OUT/tr.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
