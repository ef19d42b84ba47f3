#!/bin/bash
# round-2 GPU check: full GPU suite, smoke, default bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "host cpus: $(nproc)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench1.err; cat gpurun_out/bench1.json
exit $rc
