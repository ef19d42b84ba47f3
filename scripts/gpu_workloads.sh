#!/bin/bash
# Per-config benches (single GPU). Usage: bash scripts/gpu_workloads.sh TAG
TAG=${1:-wl}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
for w in c2 c5 c3; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail -20 $OUT/bench_$w.err; exit 1; }
  python - $OUT/bench_$w.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["config"]["workload"][:40], d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"])
print("  ", {k: v["us"] for k, v in d["kernels"].items() if v["us"] > 40})
PY
done
