#!/bin/bash
# SQ counter passes and HBM bytes over gemm_bf16_bench cases (one rocprofv3 run per pass):
#   bash scripts/pmc_bf16.sh <outdir> <case-substring>...   (each substring is also the output tag)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
for case in "$@"; do
  tag=${case// /_}
  i=0
  for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d $OUT -o ${tag}_pass$i --output-format csv -- python scripts/gemm_bf16_bench.py 5 "$case" > /dev/null 2>&1 || { echo "pmc $case pass $i failed"; exit 1; }
  done
done
echo pmc done
