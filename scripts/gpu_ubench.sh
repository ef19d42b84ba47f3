#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 ./scripts/ubench_gather.bin 26000013 3407872 > gpurun_out/ubench_gather.txt 2>&1; rc=$?
cat gpurun_out/ubench_gather.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./scripts/ubench_gather.bin 1000000 3407872 > gpurun_out/ubench_gather_small.txt 2>&1; cat gpurun_out/ubench_gather_small.txt
