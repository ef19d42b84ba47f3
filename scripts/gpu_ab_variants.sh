#!/bin/bash
# A/B of library variants on the default C2 bench, alternating: bash scripts/gpu_ab_variants.sh TAG v1 v2 ...
# ("base" = libdlamd.so; others = libdlamd_<v>.so built with DLAMD_VARIANT)
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset DLAMD_VARIANT; else export DLAMD_VARIANT=$v; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err
    rc=$?
    [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 $OUT/${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$OUT/${v}_$round.json')); k=d['kernels']
print('$v r$round ms %.4f  bwd %.1f gather %.1f fwd %.1f' % (d['ms_per_step'], k['embed_bwd']['us'], k['rec_gather']['us'], k['embed_fwd']['us']))"
  done
done
unset DLAMD_VARIANT
