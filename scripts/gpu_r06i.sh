#!/bin/bash
# round 6: two samples in flight per wave in the plain / slot lookups (SPW): kernel + parity
# suites, then the C2 bench's lookup legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-extra --no-cpu-baseline --steps 20 > $O/bench.json 2> $O/bench.log || exit $?
python - <<'PY' > $O/ab.txt
import json
d = json.loads([l for l in open("gpurun_out/r06i/bench.json") if l.strip()][-1])
g = d["gather_north_star"]["lookup_alone"]
for name, x in (("uniform", g), ("zipf", g["zipf"])):
    f = x["fused"]
    print("%s step %.4f ms | lookup %.1f us frac %.3f | fused: fm %.1f l0g %.1f l0 %.1f -> %.1f us frac %.3f pair %s" % (
        name, d["ms_per_step"], x["us"], x["frac"], f["fm_lookup_us"], f["fwd_l0_gather_us"], f["fwd_l0_plain_us"],
        f["us"], f["frac"], f["lookup_plus_l0_us"]))
PY
