#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "host cpus: $(nproc)"; rocm-smi --showproductname 2>/dev/null | head -20
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench1.err; cat gpurun_out/bench1.json
exit $rc
