#!/bin/bash
# run each argument as one GPU step (own time limit), stop at the first failure
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for c in "$@"; do
  i=$((i+1))
  echo "== [$c]"
  timeout -k 10 600 bash -c "$c" > gpurun_out/step$i.log 2>&1
  rc=$?
  tail -40 gpurun_out/step$i.log
  echo "== rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
