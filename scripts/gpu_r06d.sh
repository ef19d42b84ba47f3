#!/bin/bash
# round 6: HBM copy variants; SQ counters of the reworked bf16 NT kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 scripts/ubench_copy.hip -o /tmp/ubench_copy > /dev/null 2>&1 || exit 1
timeout -k 10 120 /tmp/ubench_copy > $O/ubench_copy.txt 2>&1 || exit $?
bash scripts/pmc_bf16.sh $O/pmc "fwd_l0 bf16 out relu" "dx_l1 mask bf16" > $O/pmc.log 2>&1 || exit $?
SQ_KERNEL=gemm_bf16_nt python scripts/sq_summary.py $O/pmc $O/bf16_nt_sq_counters.json fwd_l0_bf16_out_relu dx_l1_mask_bf16 > $O/sq.txt 2>&1
