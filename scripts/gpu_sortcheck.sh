#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -k "index or sorted or lazy" 2>&1 | tail -2 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bs.json 2>/dev/null || exit 2
python -c "import json; d=json.load(open('gpurun_out/bs.json')); print(d['value'], d['ms_per_step'], d['kernels']['index_build'])"
