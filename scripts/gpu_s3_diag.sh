#!/bin/bash
# s3 GEMM diagnostic builds (DL_S3_DIAG=1..5, libdlamd_diag<d>.so) against the default: one timed
# s3_bench case each.  bash scripts/gpu_s3_diag.sh TAG CASE
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${1:-diag}; mkdir -p $OUT
for rep in 1 2; do
  for v in "" diag1 diag2 diag3 diag4 diag5; do
    DLAMD_VARIANT=$v timeout -k 10 120 python scripts/s3_bench.py 30 t:$2 2>&1 | grep -v amdgpu.ids | sed "s/^/[${v:-default}] /" | tee -a $OUT/diag.txt || exit 1
  done
done
