#!/bin/bash
# round 6: the plain lookup's launch bound at 4 waves a SIMD (variant mw4: 100 VGPRs, no spill)
# against 5 (96 VGPRs, 3 spilled) — the full slot-plane lookup alone, then the C2 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z5
mkdir -p $O
for d in uniform zipf; do
  for v in "" mw4 "" mw4; do
    DLAMD_VARIANT=$v timeout -k 10 200 python -u scripts/lookup_bench.py $d 100 full 2>/dev/null | sed "s/^/[${v:-main}] /" >> $O/ab.txt || exit $?
  done
done
for v in "" mw4 "" mw4; do
  DLAMD_VARIANT=$v timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/c2_${v:-main}.log || exit $?
  grep "headline" $O/c2_${v:-main}.log | tail -1 | cut -c1-300 | sed "s/^/[${v:-main}] /" >> $O/ab.txt
done
cat $O/ab.txt
