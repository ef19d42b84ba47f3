#!/bin/bash
# GEMM stall breakdown: SQ counters per kernel. Usage: bash scripts/gpu_gemm_pmc.sh TAG
TAG=${1:-gpmc}
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python scripts/gemm_bench.py 20 > $OUT/gemm.txt 2>&1 || exit 1
cat $OUT/gemm.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/p1 -o p1 -- python scripts/gemm_bench.py 3 > $OUT/p1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/p2 -o p2 -- python scripts/gemm_bench.py 3 > $OUT/p2.log 2>&1 || exit 3
echo done
