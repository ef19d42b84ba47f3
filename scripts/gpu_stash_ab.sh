cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/stash
DLAMD_REC_STASH=0 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider -k lazy > gpurun_out/stash/t0.log 2>&1 || { tail -20 gpurun_out/stash/t0.log; exit 1; }
tail -1 gpurun_out/stash/t0.log
DLAMD_REC_STASH=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/stash/b0.json 2>/dev/null || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/stash/b1.json 2>/dev/null || exit 3
python - <<'PY'
import json
for f in ("b0","b1"):
    d=json.load(open("gpurun_out/stash/%s.json"%f)); k=d["kernels"]
    print(f, d["value"], d["ms_per_step"], "gather", k["rec_gather"]["us"], "bwd", k["embed_bwd"]["us"])
PY
