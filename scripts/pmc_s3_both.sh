cd "$GRAFT_REPO_ROOT"
bash scripts/pmc_s3.sh fwd_l1 && mkdir -p gpurun_out/pmc_fwd && mv gpurun_out/pmc/* gpurun_out/pmc_fwd/ && bash scripts/pmc_s3.sh dw_l1 && mkdir -p gpurun_out/pmc_dw && mv gpurun_out/pmc/* gpurun_out/pmc_dw/
