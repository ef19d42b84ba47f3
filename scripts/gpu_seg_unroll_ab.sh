cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r03u4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "hot" -p no:cacheprovider --timeout 200 --timeout-method thread 2>&1 | tail -1
for arm in new u16 new u16; do
  if [ $arm = new ]; then E="DLAMD_AB_ARM=new"; else E="DLAMD_VARIANT=u16"; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $OUT/c2_$arm.json 2>/dev/null || exit 1
  python -c "
import json;d=json.loads(open('$OUT/c2_$arm.json').read().strip().splitlines()[-1]);print('c2 $arm', d['ms_per_step'], d['kernels']['embed_bwd']['us'])"
done
for arm in new u16; do
  if [ $arm = new ]; then E="DLAMD_AB_ARM=new"; else E="DLAMD_VARIANT=u16"; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --dist zipf --workload c3 --steps 10 --warmup 3 > $OUT/c3z_$arm.json 2>/dev/null || exit 1
  python -c "
import json;d=json.loads(open('$OUT/c3z_$arm.json').read().strip().splitlines()[-1]);print('c3 zipf $arm', d['ms_per_step'], d['kernels']['embed_bwd']['us'])"
done
