#!/bin/bash
# Final-tree evidence: GPU suite, the full-size trajectories, smoke, the default bench line, the
# C3 / C5 lines and rocprofv3 stats of the C2 bench: bash scripts/gpu_final.sh TAG
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; mkdir -p $OUT
bash scripts/gpu_r05.sh $1 suite fullsize smoke || exit $?
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
tail -c 600 $OUT/bench_default.json; echo
for wl in c3 c5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -5 $OUT/bench_$wl.err; exit 1; }
  python -c "
import json;d=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$wl', d['ms_per_step'], {n: k[n]['us'] for n in k})"
done
bash scripts/prof_stats.sh $1/rocprof_c2 python bench.py --no-cpu-baseline --no-extra --steps 20 > $OUT/rocprof_c2.txt 2>&1; cat $OUT/rocprof_c2.txt | head -12
