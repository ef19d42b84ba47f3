#!/bin/bash
# round 6: predict's front, unfused (lookup + plain first layer) and fused (FM-only lookup +
# the gathering first layer): time, rocprofv3 stats and PMC passes (uniform, Zipf)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m
bash scripts/gpu_lookup_pmc.sh r06m/pair pair > gpurun_out/r06m/pair.txt 2>&1 || exit $?
bash scripts/gpu_lookup_pmc.sh r06m/fused fused > gpurun_out/r06m/fused.txt 2>&1
