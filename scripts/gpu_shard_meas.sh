cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/shm; mkdir -p $OUT
run() { local n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; return 1; }
  python -c "
import json;d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n', d['ms_per_step'], {x: k[x]['us'] for x in k})"; }
run c2 --steps 20 --warmup 5 && run c2_sharded1 --sharded --vocab 1000000 --steps 20 --warmup 5 && run c2_sharded1_chain --sharded --vocab 1000000 --owner-update chain --steps 20 --warmup 5 && run c5_nopf --workload c5 --no-prefetch --steps 20 --warmup 5 && run c5 --workload c5 --steps 20 --warmup 5
