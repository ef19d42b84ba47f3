#!/bin/bash
# round 6: the lookups' x0 cont columns from the tile's staged values (no per-sample HBM round
# trip): kernel + parity suites, then the C2 bench lookup legs, default vs two samples a wave
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
for v in "" spw2 "" spw2; do
  DLAMD_VARIANT=$v timeout -k 10 600 python -u bench.py --no-extra --no-cpu-baseline --steps 20 > $O/bench_${v:-main}.json 2>> $O/bench_${v:-main}.log || exit $?
  python - "$O/bench_${v:-main}.json" "${v:-main}" >> $O/ab.txt <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.strip()][-1])
g = d["gather_north_star"]["lookup_alone"]
k = d["kernels"]
for name, x in (("uniform", g), ("zipf", g["zipf"])):
    f = x["fused"]
    print("%-5s %-7s step %.4f ms embed_fwd %.1f | lookup %.1f us frac %.3f | fused: fm %.1f l0g %.1f l0 %.1f -> %.1f us frac %.3f pair %s" % (
        sys.argv[2], name, d["ms_per_step"], k["embed_fwd"]["us"], x["us"], x["frac"], f["fm_lookup_us"],
        f["fwd_l0_gather_us"], f["fwd_l0_plain_us"], f["us"], f["frac"], f["lookup_plus_l0_us"]))
PY
done
