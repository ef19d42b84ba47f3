#!/bin/bash
# round 6: the FM-only lookup of the fused predict — time, stats and PMC passes (uniform, Zipf)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06j
bash scripts/gpu_lookup_pmc.sh r06j fm > gpurun_out/r06j/run.txt 2>&1
