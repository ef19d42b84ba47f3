#!/bin/bash
# GEMM iteration: kernel tests + one parity case + lazy bench. Usage: bash scripts/gpu_gemm.sh TAG
TAG=${1:-gemm}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "gemm or (deepfm_pipeline and 1536 and lazy)" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --adam lazy > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 $OUT/bench.err
python - $OUT/bench.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"])
for k,v in d["kernels"].items():
    if "gemm" in k: print(k, v["us"], v.get("frac_mfma"))
PY
exit $rc
