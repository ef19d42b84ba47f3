#!/bin/bash
# SQ counter passes over s3_bench cases (one rocprofv3 run per pass): bash scripts/pmc_s3.sh <outdir> case...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
for case in "$@"; do
  i=0
  for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT -o ${case}_pass$i --output-format csv -- python scripts/s3_bench.py 5 $case > /dev/null 2>&1 || { echo "pmc $case pass $i failed"; exit 1; }
  done
done
echo pmc done
