#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python scripts/diag_race.py 65536 12 > gpurun_out/race.out 2>&1; rc=$?
cat gpurun_out/race.out | grep -v amdgpu.ids; exit $rc
