#!/bin/bash
# round 6: fused-gather A/B — natural k order (default), the k-permuted planes (DL_S3_KPERM:
# a wave instruction reads whole 64-B rows), and the row-0 diagnostics build (the gather's
# memory cost); the kperm build's gather / s3 tests first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
DLAMD_VARIANT=kperm timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "gather or flat_lookup or s3" > $O/pytest_kperm.log 2>&1 || exit $?
for v in "" kperm gdiag "" kperm; do
  DLAMD_VARIANT=$v timeout -k 10 600 python -u bench.py --no-extra --no-cpu-baseline --steps 20 > $O/bench_${v:-main}.json 2>> $O/bench_${v:-main}.log || exit $?
  python - "$O/bench_${v:-main}.json" "${v:-main}" >> $O/ab.txt <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.strip()]
d = json.loads(lines[-1])
g = d["gather_north_star"]["lookup_alone"]
f, z = g["fused"], g["zipf"]["fused"]
print("%-6s step %.4f ms | uniform fm %.1f l0g %.1f l0 %.1f -> %.1f us frac %.3f pair %s | zipf fm %.1f l0g %.1f l0 %.1f -> %.1f us frac %.3f pair %s" % (
    sys.argv[2], d["ms_per_step"], f["fm_lookup_us"], f["fwd_l0_gather_us"], f["fwd_l0_plain_us"], f["us"], f["frac"],
    f["lookup_plus_l0_us"], z["fm_lookup_us"], z["fwd_l0_gather_us"], z["fwd_l0_plain_us"], z["us"], z["frac"],
    z["lookup_plus_l0_us"]))
PY
done
