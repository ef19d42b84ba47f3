#!/bin/bash
# selected GPU tests ($1, or "none"), then one bench run per remaining argument (quoted bench flags)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
sel="$1"; shift
if [ "$sel" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 600 --timeout-method thread -k "$sel" > gpurun_out/pytest_sel.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py $a > gpurun_out/ab$i.json 2> gpurun_out/ab$i.err
  rc=$?
  echo "== bench [$a] rc=$rc"; tail -3 gpurun_out/ab$i.err
  python -c "
import json,sys; d=json.load(open('gpurun_out/ab$i.json')); k=d['kernels']
print('value %.3fM ms %.3f roof %s %.3f' % (d['value']/1e6, d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))
print(' '.join('%s=%.0f' % (n, v['us']) for n, v in k.items()))
print('cpu', d.get('cpu_baseline')); print('gather', d.get('gather_north_star'), 'flush', d.get('table_flush'))" || true
  [ $rc -eq 0 ] || exit $rc
done
