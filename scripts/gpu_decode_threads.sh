#!/bin/bash
# Drop-in loop with the native decoder's thread team at several sizes (DLIO_DECODE_THREADS), after
# the drop-in GPU tests:  bash scripts/gpu_decode_threads.sh TAG "threads..."
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -k "dropin or native_pickle" -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_dropin.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_dropin.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for t in $2; do
    DLIO_DECODE_THREADS=$t timeout -k 10 300 python scripts/dropin_feed_timing.py 24 > $OUT/feed_t${t}_$rep.log 2>&1 || { tail -5 $OUT/feed_t${t}_$rep.log; exit 1; }
    echo "threads=$t $(grep ms/step $OUT/feed_t${t}_$rep.log | tail -1)" | tee -a $OUT/decode_threads.txt
  done
done
