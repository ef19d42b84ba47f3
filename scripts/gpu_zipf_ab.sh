#!/bin/bash
# Zipf-id bench arms (C3, C2) of the default library against a variant: bash scripts/gpu_zipf_ab.sh TAG VAR "<-k>"
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; VAR=$2; mkdir -p $OUT
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -k "$3" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_k.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_k.log | head -20; exit $rc; }
fi
for wl in c3 c2; do
  for arm in new $VAR; do
    if [ $arm = new ]; then E="DLAMD_AB_ARM=new"; else E="DLAMD_VARIANT=$VAR"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --dist zipf --workload $wl --steps 10 --warmup 3 > $OUT/zipf_${wl}_$arm.json 2> $OUT/zipf_${wl}_$arm.err || { tail -5 $OUT/zipf_${wl}_$arm.err; exit 1; }
    python -c "
import json;d=json.loads(open('$OUT/zipf_${wl}_$arm.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$wl $arm', d['ms_per_step'], {n: k[n]['us'] for n in ('embed_bwd', 'rec_gather', 'index_build') if n in k})"
  done
done
