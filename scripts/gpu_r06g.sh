#!/bin/bash
# round 6: the deep lookup fused into the first tower layer (dl_gemm_s3_nt_gather): kernel and
# predict bit-identity tests, then the C2 bench's lookup legs (plain and fused, uniform and Zipf)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "gather or flat_lookup" > $O/pytest_gather.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-extra --no-cpu-baseline --steps 20 > $O/bench.json 2> $O/bench.log || exit $?
python - <<'PY' > $O/gather.txt
import json
d = json.load(open("gpurun_out/r06g/bench.json"))
g = d.get("gather_north_star") or {}
print(json.dumps(g, indent=1))
PY
