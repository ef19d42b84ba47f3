#!/bin/bash
# round 6: the training forward's deep rows gathered by the first s3 layer (default) against the
# indexed lookup writing x0 (DLAMD_FUSED_GATHER=0): C2, C3 and C2 Zipf steps A/B on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
for a in 1 0 1 0; do
  for wl in c2 c3; do
    DLAMD_FUSED_GATHER=$a timeout -k 10 300 python -u bench.py --workload $wl --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/${wl}_$a.log || exit $?
    grep "headline" $O/${wl}_$a.log | tail -1 | cut -c1-400 | sed "s/^/[fused=$a] /" >> $O/ab.txt
  done
  DLAMD_FUSED_GATHER=$a timeout -k 10 300 python -u bench.py --dist zipf --no-extra --no-cpu-baseline --steps 30 > /dev/null 2>> $O/c2z_$a.log || exit $?
  grep "headline" $O/c2z_$a.log | tail -1 | cut -c1-400 | sed "s/^/[fused=$a zipf] /" >> $O/ab.txt
done
